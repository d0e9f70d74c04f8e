// vg_dev.h — device-side helpers shared by the map, IEKF and BA kernels.
#pragma once
#include "vg_internal.h"

namespace vg {

__device__ __forceinline__ M3 ld_m3(const double* a) {
  M3 m;
  for (int i = 0; i < 9; i++) m[i] = a[i];
  return m;
}
__device__ __forceinline__ V3 ld_v3(const double* a) { return v3(a[0], a[1], a[2]); }

// voxel key rule for double coordinates (voxel_map.cpp:57-65, 246-253)
__device__ __forceinline__ int64_t key_axis_d(double c, double size) {
  float l = (float)(c / size);
  if (l < 0) l -= 1;
  return (int64_t)l;
}
__device__ __forceinline__ bool pack_key(const V3& w, double size, uint64_t& out) {
  int64_t k[3];
  bool ok = true;
  for (int j = 0; j < 3; j++) {
    k[j] = key_axis_d(w[j], size) + kKeyOff;
    ok &= (k[j] >= 0) & (k[j] < 2 * kKeyOff);
  }
  out = ok ? (((uint64_t)k[0] << 42) | ((uint64_t)k[1] << 21) | (uint64_t)k[2]) : 0;
  return ok;
}
__device__ __forceinline__ int64_t unpack_axis(uint64_t key, int sh) {
  return (int64_t)((key >> sh) & ((1ull << 21) - 1)) - kKeyOff;
}
__device__ __forceinline__ uint32_t hash_slot(uint64_t k, int mask) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return (uint32_t)k & (uint32_t)mask;
}
// open-addressing lookup of a root voxel: node id or -1
__device__ __forceinline__ int hash_find(const uint64_t* __restrict__ hkey, const int* __restrict__ hval, int mask,
                                         uint64_t key) {
  uint32_t s = hash_slot(key, mask);
  for (int probe = 0; probe <= mask; probe++) {
    uint64_t k = hkey[s];
    if (k == key) return hval[s];
    if (k == kKeyEmpty) return -1;
    s = (s + 1) & (uint32_t)mask;
  }
  return -1;
}
// insert-or-find; returns the slot, sets fresh if this thread inserted the key
__device__ __forceinline__ int hash_insert(uint64_t* hkey, int mask, uint64_t key, bool& fresh) {
  uint32_t s = hash_slot(key, mask);
  fresh = false;
  for (int probe = 0; probe <= mask; probe++) {
    unsigned long long prev = atomicCAS((unsigned long long*)&hkey[s], (unsigned long long)kKeyEmpty,
                                        (unsigned long long)key);
    if (prev == kKeyEmpty) {
      fresh = true;
      return (int)s;
    }
    if (prev == key) return (int)s;
    s = (s + 1) & (uint32_t)mask;
  }
  return -1;
}

// owner rank of a 16^3-root-voxel tile given by its coordinates (the offset
// voxel key >> 4 per axis)
__host__ __device__ __forceinline__ int tile_owner_t(uint64_t tx, uint64_t ty, uint64_t tz, int world) {
  uint64_t h = (tx * 0x9E3779B97F4A7C15ull) ^ (ty * 0xC2B2AE3D27D4EB4Full) ^ (tz * 0x165667B19E3779F9ull);
  h ^= h >> 31;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 29;
  return (int)(h % (uint64_t)world);
}
// of the tile holding a packed root key (oracle/map.hpp tile_owner is the same function)
__host__ __device__ __forceinline__ int tile_owner(uint64_t key, int world) {
  return tile_owner_t((key >> 46) & 0x1ffff, (key >> 25) & 0x1ffff, (key >> 4) & 0x1ffff, world);
}
// Sharded mode's keep list (DState::skeep, map.hip k_keep_*): usable while the
// current pose x_curr moved every point by less than kmargin from the pose the
// list was made at — |dR|_2 r_max + |dp| bounds |R q + p - (R0 q + p0)| for
// |q| <= r_max, and for two rotations |R - R0|_2 = |R - R0|_F / sqrt(2) (the
// singular values of R0 (Q - I) are 2 sin(a/2) twice and 0; 1.4 leaves room for
// rounding). Every lane of every IEKF kernel evaluates it on the same state.
__device__ __forceinline__ const int* iekf_keep(const DState* __restrict__ st) {
  const int* k = st->skeep;
  if (!k) return nullptr;
  double dr = 0.0, dp = 0.0;
  for (int t = 0; t < 9; t++) {
    const double d = st->xc[t] - st->kpose[t];
    dr += d * d;
  }
  for (int t = 9; t < 12; t++) {
    const double d = st->xc[t] - st->kpose[t];
    dp += d * d;
  }
  return sqrt(dr) * (1.0 / 1.4) * st->krmax + sqrt(dp) < st->kmargin ? k : nullptr;
}
// the points the IEKF point loop takes this iteration
__device__ __forceinline__ int iekf_n(const DState* __restrict__ st) { return iekf_keep(st) ? st->snk : st->sn; }
__device__ __forceinline__ bool owns(const DevMap& m, uint64_t key) {
  return m.shard_world <= 1 || tile_owner(key, m.shard_world) == m.shard_rank;
}
// the thread_num quirks (voxel_map.cpp:96-97, local_mapping.cpp:27, 93, 150)
// compare GLOBAL counts: the all-reduced copies in sharded mode
__device__ __forceinline__ int g_touched(const DevMap& m) {
  return m.shard_world > 1 ? m.counters[kCntGTouched] : m.counters[kCntTouched];
}
__device__ __forceinline__ int g_slide(const DevMap& m) {
  return m.shard_world > 1 ? m.counters[kCntGSlide] : m.counters[kCntSlide];
}

__device__ __forceinline__ int octant(const V3& p, const double* c) {
  return 4 * (p[0] > c[0] ? 1 : 0) + 2 * (p[1] > c[1] ? 1 : 0) + (p[2] > c[2] ? 1 : 0);
}

// calcBodyVar — point_utils.cpp:3-34 (modifies pb[2] when 0, like the reference)
// dv = sin^2(degree_inc * pi / 180) is a per-configuration constant, computed
// once on the host (MP::beam_dv) instead of one fp64 sin per point
__device__ __forceinline__ M3 calc_body_var(V3& pb, float range_inc, double dv) {
  if (pb[2] == 0) pb[2] = 0.0001;
  float range = sqrt(pb[0] * pb[0] + pb[1] * pb[1] + pb[2] * pb[2]);
  float range_var = range_inc * range_inc;
  double nb = norm3(pb);
  V3 d = v3(pb[0] / nb, pb[1] / nb, pb[2] / nb);
  M3 dhat = hat(d);
  V3 b1 = v3(1, 1, -(d[0] + d[1]) / d[2]);
  double n1 = norm3(b1);
  b1 = v3(b1[0] / n1, b1[1] / n1, b1[2] / n1);
  V3 b2 = cross3(b1, d);
  double n2 = norm3(b2);
  b2 = v3(b2[0] / n2, b2[1] / n2, b2[2] / n2);
  M<3, 2> Nm;
  Nm(0, 0) = b1[0]; Nm(0, 1) = b2[0];
  Nm(1, 0) = b1[1]; Nm(1, 1) = b2[1];
  Nm(2, 0) = b1[2]; Nm(2, 1) = b2[2];
  M<3, 2> A = mul(scl(dhat, (double)range), Nm);
  M<2, 2> D;
  D.zero();
  D(0, 0) = dv;
  D(1, 1) = dv;
  V3 dr = v3(d[0] * (double)range_var, d[1] * (double)range_var, d[2] * (double)range_var);
  return add(outer3(dr, d), mul(mul(A, D), tr(A)));
}

// var_init (point_utils.cpp:36-52) for one raw point: body pnt (after the
// extrinsic) and its covariance.
__device__ __forceinline__ void var_init_pt(const MP& mp, float x, float y, float z, V3& pnt, M3& var) {
  V3 pb = v3(x, y, z);
  M3 vb = calc_body_var(pb, mp.dept, mp.beam_dv);
  M3 eR = ld_m3(mp.extR);
  pnt = rigid(eR, pb, ld_v3(mp.extt));
  var = mul(mul(eR, vb), tr(eR));
}

// pvec_update world covariance (point_utils.cpp:60): R v R^T + [p] S_R [p]^T + S_t
__device__ __forceinline__ M3 world_var(const M3& R, const M3& var, const V3& pnt, const M3& rot_var,
                                        const M3& tsl_var) {
  M3 ph = hat(pnt);
  return add(add(mul(mul(R, var), tr(R)), mul(mul(ph, rot_var), tr(ph))), tsl_var);
}

// cov_add += Bf_var(pv, vec) (octree.cpp:83-92) on packed upper 9x9.
// Bi has 9 non-zeros; Bu = Bi*var and Bu*Bi^T are expanded with the zero terms
// dropped (same non-zero term order as the dense product, so every sum is
// bit-identical to it) to keep the accumulator in registers.
__device__ __forceinline__ void bf_var_acc(double* __restrict__ cov, const M3& V, const V3& p) {
  const double x = p[0], y = p[1], z = p[2];
  const double x2 = 2 * x, y2 = 2 * y, z2 = 2 * z;
  double Bu[6][3];
  for (int c = 0; c < 3; c++) {
    Bu[0][c] = x2 * V(0, c);
    Bu[1][c] = y * V(0, c) + x * V(1, c);
    Bu[2][c] = z * V(0, c) + x * V(2, c);
    Bu[3][c] = y2 * V(1, c);
    Bu[4][c] = z * V(1, c) + y * V(2, c);
    Bu[5][c] = z2 * V(2, c);
  }
  // B66(r, c) = sum_k Bu(r,k) Bi(c,k), Bi rows: [2x,0,0] [y,x,0] [z,0,x] [0,2y,0] [0,z,y] [0,0,2z]
  int k = 0;
#pragma unroll
  for (int r = 0; r < 6; r++) {
    const double b0 = Bu[r][0], b1 = Bu[r][1], b2 = Bu[r][2];
    const double col[6] = {b0 * x2, b0 * y + b1 * x, b0 * z + b2 * x, b1 * y2, b1 * z + b2 * y, b2 * z2};
#pragma unroll
    for (int c = 0; c < 6; c++)
      if (c >= r) cov[k++] += col[c];
#pragma unroll
    for (int c = 0; c < 3; c++) cov[k++] += Bu[r][c];
  }
  cov[k++] += V(0, 0);
  cov[k++] += V(0, 1);
  cov[k++] += V(0, 2);
  cov[k++] += V(1, 1);
  cov[k++] += V(1, 2);
  cov[k++] += V(2, 2);
}

// ---- wave-cooperative ordered accumulation --------------------------------
// A leaf's running sums (clusters, cov_add) are order-dependent in rounding.
// Instead of one thread walking a leaf's points (one dependent load chain per
// point), a whole wave takes the leaf: lanes prefetch 64 point records into
// LDS at a time, and each lane owns one running sum, applying every point in
// order. Every increment is written as
//   (E[i1] E[i2] + E[i3] E[i4]) E[i5] + (E[i6] E[i7] + E[i8] E[i9]) E[i10]
// over the point record E, with operand slots chosen per lane; the unused
// slots read 0 or 1, which leaves every rounding step of clu_push and
// bf_var_acc unchanged (x + 0 = x, x * 1 = x).
enum { kEq = 0, kEp = 3, kEv = 6, kEx2 = 15, kEy2 = 16, kEz2 = 17, kEone = 18, kEzero = 19, kErec = 20 };
struct RoleIdx {
  unsigned char i[10];
};

// point record: q = cluster-local point, p = world point (add / cov), V = var
__device__ __forceinline__ void fill_record(double* E, const V3& q, const V3& p, const M3& V) {
  for (int t = 0; t < 3; t++) {
    E[kEq + t] = q[t];
    E[kEp + t] = p[t];
  }
  for (int t = 0; t < 9; t++) E[kEv + t] = V[t];
  E[kEx2] = 2 * p[0];
  E[kEy2] = 2 * p[1];
  E[kEz2] = 2 * p[2];
  E[kEone] = 1.0;
  E[kEzero] = 0.0;
}

__device__ __forceinline__ RoleIdx role_make(int i1, int i2, int i3, int i4, int i5, int i6 = kEzero,
                                             int i7 = kEzero, int i8 = kEzero, int i9 = kEzero, int i10 = kEone) {
  RoleIdx r;
  r.i[0] = i1; r.i[1] = i2; r.i[2] = i3; r.i[3] = i4; r.i[4] = i5;
  r.i[5] = i6; r.i[6] = i7; r.i[7] = i8; r.i[8] = i9; r.i[9] = i10;
  return r;
}

// clu_push component (P0..P5 = xx xy xz yy yz zz, then v0..v2) of the point at `base`
__device__ __forceinline__ RoleIdx role_clu(int comp, int base) {
  const int a[6] = {0, 0, 0, 1, 1, 2}, b[6] = {0, 1, 2, 1, 2, 2};
  if (comp < 6) return role_make(base + a[comp], base + b[comp], kEzero, kEzero, kEone);
  return role_make(base + comp - 6, kEone, kEzero, kEzero, kEone);
}

// Bu(r, c) of bf_var_acc as (i1, i2, i3, i4)
__device__ __forceinline__ void bu_ops(int r, int c, int* o) {
  const int X = kEp, Y = kEp + 1, Z = kEp + 2;
  auto V = [](int a, int cc) { return kEv + 3 * a + cc; };
  switch (r) {
    case 0: o[0] = kEx2; o[1] = V(0, c); o[2] = kEzero; o[3] = kEzero; break;
    case 1: o[0] = Y; o[1] = V(0, c); o[2] = X; o[3] = V(1, c); break;
    case 2: o[0] = Z; o[1] = V(0, c); o[2] = X; o[3] = V(2, c); break;
    case 3: o[0] = kEy2; o[1] = V(1, c); o[2] = kEzero; o[3] = kEzero; break;
    case 4: o[0] = Z; o[1] = V(1, c); o[2] = Y; o[3] = V(2, c); break;
    default: o[0] = kEz2; o[1] = V(2, c); o[2] = kEzero; o[3] = kEzero; break;
  }
}

// cov_add entry k (0..44) in bf_var_acc's order
__device__ __forceinline__ RoleIdx role_cov(int k) {
  const int X = kEp, Y = kEp + 1, Z = kEp + 2;
  int q = 0;
  for (int r = 0; r < 6; r++) {
    for (int c = r; c < 6; c++, q++) {
      if (q != k) continue;
      // col[c] = bA * s + bB * t  (b0, b1, b2 = Bu(r, 0..2))
      const int ca[6] = {0, 0, 0, 1, 1, 2}, cs[6] = {kEx2, Y, Z, kEy2, Z, kEz2};
      const int cb[6] = {-1, 1, 2, -1, 2, -1}, ct[6] = {kEone, X, X, kEone, Y, kEone};
      int A[4], B[4] = {kEzero, kEzero, kEzero, kEzero};
      bu_ops(r, ca[c], A);
      if (cb[c] >= 0) bu_ops(r, cb[c], B);
      return role_make(A[0], A[1], A[2], A[3], cs[c], B[0], B[1], B[2], B[3], ct[c]);
    }
    for (int c = 0; c < 3; c++, q++) {
      if (q != k) continue;
      int A[4];
      bu_ops(r, c, A);
      return role_make(A[0], A[1], A[2], A[3], kEone);
    }
  }
  const int va[6] = {0, 0, 0, 1, 1, 2}, vb[6] = {0, 1, 2, 1, 2, 2};
  const int j = k - q;
  return role_make(kEv + 3 * va[j] + vb[j], kEone, kEzero, kEzero, kEone);
}

__device__ __forceinline__ double role_inc(const double* E, const RoleIdx& r) {
  const double A = E[r.i[0]] * E[r.i[1]] + E[r.i[2]] * E[r.i[3]];
  const double B = E[r.i[5]] * E[r.i[6]] + E[r.i[7]] * E[r.i[8]];
  return A * E[r.i[4]] + B * E[r.i[9]];
}

// Wave-aggregated append: every lane of the wave must call it (uniform control
// flow); returns this lane's first slot. One atomic per wave instead of one per
// element (a single hot counter serialises at ~88 ops/us, MI355X_MICROARCH
// 'dequeue').
// a leaf's run of window points in one physical slot (DevMap::lseg)
__device__ __forceinline__ uint64_t lseg_pack(int start, int count, int epoch) {
  return (uint64_t)(start & 0xffffff) | ((uint64_t)(count & 0x1fffff) << 24) | ((uint64_t)(epoch & 0x7ffff) << 45);
}
__device__ __forceinline__ bool lseg_get(const DevMap& m, int leaf, int slot, int& start, int& count) {
  const uint64_t v = m.lseg[(size_t)leaf * m.W + slot];
  start = (int)(v & 0xffffff);
  count = (int)((v >> 24) & 0x1fffff);
  return count > 0 && (int)(v >> 45) == (m.slot_epoch[slot] & 0x7ffff);
}

__device__ __forceinline__ int wave_append(int* ctr, int count) {
  const int lane = threadIdx.x & 63;
  int x = count;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  const int total = __shfl(x, 63, 64);
  int base = 0;
  if (lane == 63 && total > 0) base = atomicAdd(ctr, total);
  base = __shfl(base, 63, 64);
  return base + x - count;
}

// three wave appends at once: one scan of the counts packed 21 bits each
// (every count < 2^21 / 64), the three atomics issued back to back
__device__ __forceinline__ void wave_append3(int* c0, int n0, int* c1, int n1, int* c2, int n2, int& o0, int& o1,
                                             int& o2) {
  const int lane = threadIdx.x & 63;
  const unsigned long long v = (unsigned long long)n0 | ((unsigned long long)n1 << 21) | ((unsigned long long)n2 << 42);
  unsigned long long x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  const unsigned long long tot = __shfl(x, 63, 64);
  const int t0 = (int)(tot & 0x1fffff), t1 = (int)((tot >> 21) & 0x1fffff), t2 = (int)(tot >> 42);
  int b0 = 0, b1 = 0, b2 = 0;
  if (lane == 63) {
    if (t0 > 0) b0 = atomicAdd(c0, t0);
    if (t1 > 0) b1 = atomicAdd(c1, t1);
    if (t2 > 0) b2 = atomicAdd(c2, t2);
  }
  const unsigned long long ex = x - v;
  o0 = __shfl(b0, 63, 64) + (int)(ex & 0x1fffff);
  o1 = __shfl(b1, 63, 64) + (int)((ex >> 21) & 0x1fffff);
  o2 = __shfl(b2, 63, 64) + (int)(ex >> 42);
}

__device__ __forceinline__ M<9, 9> unpack9(const double* cov) {
  M<9, 9> m;
  int k = 0;
  for (int r = 0; r < 9; r++)
    for (int c = r; c < 9; c++, k++) {
      m(r, c) = cov[k];
      m(c, r) = cov[k];
    }
  return m;
}

// The region the correspondence descent (octant(): w > centre takes the upper
// child, octree.cpp:586) assigns to a node: lo < w <= hi per axis, the bounds
// being ancestors' centres (roots unbounded: their membership is the float
// voxel key). The IEKF's memo of an unmatched point's leaf is valid exactly
// while the point stays in it (k_iekf); OctoTree::inside's inclusive box
// (octree.cpp:732-737) is the test for the reference's own octos[i] only.
__device__ __forceinline__ void dbox_root(double* b) {
  for (int j = 0; j < 3; j++) {
    b[j] = -__builtin_huge_val();
    b[3 + j] = __builtin_huge_val();
  }
}
__device__ __forceinline__ void dbox_child(double* b, const double* pb, const double* pc, int o) {
  for (int j = 0; j < 3; j++) {
    const bool up = (o >> (2 - j)) & 1;
    b[j] = up ? pc[j] : pb[j];
    b[3 + j] = up ? pb[3 + j] : pc[j];
  }
}
__device__ __forceinline__ bool in_dbox(const double* b, const V3& w) {
  return w[0] > b[0] && w[0] <= b[3] && w[1] > b[1] && w[1] <= b[4] && w[2] > b[2] && w[2] <= b[5];
}

__device__ __forceinline__ void init_node(NodeHdr& h, const double c[3], float qlen, int layer, int parent) {
  for (int j = 0; j < 3; j++) h.center[j] = c[j];
  for (int j = 0; j < 8; j++) h.child[j] = -1;
  h.qlen = qlen;
  h.layer = (int8_t)layer;
  h.octo = 0;
  h.isexist = 0;
  h.is_plane = 0;
  h.has_sw = 0;
  h.pad0 = h.pad1 = h.pad2 = 0;
  h.opt_state = -1;
  h.last_num = 0;
  h.fix_off = 0;
  h.fix_cnt = 0;
  h.fix_cap = 0;
  h.parent = parent;
}

// x_buf.push_back(x_curr) at ord and a fresh IMU_PRE record with zero bias
// deltas (local_mapping.cpp:434-441, imu_preintegration.cpp:10-29); one
// workgroup (k_push_state, or block 0 of k_ins_prep)
__device__ __forceinline__ void push_state_block(DState* __restrict__ st, const PushArg& pa) {
  const int t = threadIdx.x;
  if (t < kXS) st->xs[pa.ord * kXS + t] = st->xc[t];
  if (pa.new_imu >= 0) {
    if (t < 12) st->bias[pa.new_imu * 12 + t] = 0.0;
    double* d = &st->imurec[(size_t)((st->imu_head + pa.new_imu) % kMaxWin) * kBaImuRec];
    for (int e = t; e < kBaImuRec; e += blockDim.x) d[e] = pa.rec[e];
  }
}

// host-mapped publication stores. Every payload word is a system-scope store
// (written through the L2 to host memory), so ordering them before the flag
// needs no L2 write-back: each storing wave drains its stores (pub_drain, an
// s_waitcnt vmcnt(0), before the workgroup barrier), then one lane stores
// the flag, also system scope. (A system-scope release or __threadfence_system
// would write back every dirty line of the XCD's L2 first: nothing the host
// reads lives there.)
__device__ __forceinline__ void pub_store(double* dst, double v) {
  __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void pub_store(int* dst, int v) {
  __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// (gfx9 counts stores in vmcnt; gfx10+ counts them in vscnt, where this wait
// would not order the payload before the flag)
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "pub_drain orders stores with vmcnt: gfx9 (gfx950) only"
#endif
__device__ __forceinline__ void pub_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void pub_flag(int* dst, int v) {
  pub_drain();  // this wave's own payload stores
  __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// P1: x_curr, the post-IEKF pose, window states, IEKF / BA summary.
// head_flag: x_curr is final (the caller stored R/p): the next scan's device
// propagation may start (vg_ctx::d_sync[2]) — raised once what it overwrites
// (x_curr, the IEKF summary) is read, before the slow host-memory stores
__device__ __forceinline__ void publish_state_block(const DState* __restrict__ st, int win_count, int ba_iters_valid,
                                                    const int* __restrict__ ba_iters, const int* __restrict__ ba_hess,
                                                    Pub* __restrict__ pub, int seq, unsigned* head_flag = nullptr,
                                                    unsigned head_value = 0) {
  const int t = threadIdx.x;
  __shared__ double s_xc[kXC];
  __shared__ int s_sum[10];
  for (int e = t; e < kXC; e += blockDim.x) s_xc[e] = st->xc[e];
  if (t == 0) {
    s_sum[0] = st->iters;
    s_sum[9] = st->iekf_pts;
    for (int k = 0; k < 4; k++) {
      s_sum[1 + k] = st->matches[k];
      s_sum[5 + k] = st->planes[k];
    }
  }
  __syncthreads();
  if (head_flag) {
    __threadfence();
    __syncthreads();
    if (t == 0) __hip_atomic_store(head_flag, head_value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (seq <= 0) return;
  for (int e = t; e < kXC; e += blockDim.x) pub_store(&pub->xc[e], s_xc[e]);
  for (int e = t; e < 12; e += blockDim.x) pub_store(&pub->traj[e], st->traj[e]);
  for (int e = t; e < 6; e += blockDim.x) pub_store(&pub->nnt[e], st->nnt[e]);
  for (int e = t; e < win_count * kXS; e += blockDim.x) pub_store(&pub->xs[e], st->xs[e]);
  if (t == 0) {
    pub_store(&pub->iekf_iters, s_sum[0]);
    for (int k = 0; k < 4; k++) pub_store(&pub->matches[k], s_sum[1 + k]);
    pub_store(&pub->ba_iters1, ba_iters_valid ? *ba_iters : 0);
    pub_store(&pub->ba_hess1, ba_iters_valid ? *ba_hess : 0);
    for (int k = 0; k < 4; k++) pub_store(&pub->planes[k], s_sum[5 + k]);
    pub_store(&pub->iekf_pts, s_sum[9]);
  }
  pub_drain();
  __syncthreads();
  if (t == 0) pub_flag(&pub->seq1, seq);
}
// window view for the map kernels: poses by ord, ring, per-ord counts / slots
__device__ __forceinline__ void make_win_block(DState* __restrict__ st, const WinArg& wa, const int* __restrict__ wpn,
                                               WinD* __restrict__ win, int* __restrict__ nper,
                                               int* __restrict__ slot_of) {
  const int t = threadIdx.x;
  const int wc = wa.win_count;
  if (wa.set_xc && wc > 0) {
    if (t < 12) st->xc[t] = st->xs[(wc - 1) * kXS + t];
    __syncthreads();
  }
  for (int e = t; e < kMaxWin * 12; e += blockDim.x) {
    const int i = e / 12, k = e % 12;
    const double v = i < wc ? st->xs[i * kXS + k] : 0.0;
    if (k < 9) win->R[i][k] = v;
    else win->p[i][k - 9] = v;
  }
  if (t < kMaxWin) {
    win->mp[t] = wa.mp[t];
    nper[t] = t < wc ? wpn[wa.mp[t]] : 0;  // the inserts' counts (device: no host round trip)
    slot_of[t] = wa.mp[t];
  }
  if (t == 0) {  // the window's point total (the recut's window-event grid reads it)
    int tot = 0;
    for (int k = 0; k < wc && k < kMaxWin; k++) tot += wpn[wa.mp[k]];
    nper[64] = tot;
  }
  if (t == 0) {
    win->win_count = wc;
    win->pad = 0;
    st->seq2 = wa.seq2;
    if (wa.set_xc) st->jour_check = wa.jour_check;  // the margi head (k_slide_compact reads it)
  }
}
// exclusive prefix over one value per thread of a 1024-lane workgroup
__device__ __forceinline__ int block_excl_scan(int v, int* s_wsum, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_wsum[wv] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); k++) {
      int t = s_wsum[k];
      s_wsum[k] = acc;
      acc += t;
    }
    s_wsum[16] = acc;
  }
  __syncthreads();
  const int r = s_wsum[wv] + x - v;
  *total = s_wsum[16];
  __syncthreads();
  return r;
}


// the recut / margi device-side counts (Work::rc)
enum { kRcLvl = 0, kRcSub = 16, kRcWin = 32, kRcAbort = 48, kRcCh = 64, kRcChBase = 80, kRcNch = 96, kRcTot = 104,
       kRcNode0 = 112, kRcStatus = 126, kRcNOld = 127, kRcN = 128 };

// tras_opt's factor list (octree.cpp:491-516): the candidate bitmap over node
// ids -> the id-ascending factor list, cleared as it is read; the recut status
// (kRcBig: more factors than the device list holds) and the factor count
// published. One workgroup (k_fac_sort)
constexpr int kFacMax = 1 << 20;
constexpr int kRcBig = 200;
__device__ __forceinline__ void fac_sort_block(DevMap& m, int* __restrict__ rc, uint32_t* __restrict__ bits,
                                               int* __restrict__ fac_node, int cap_f, Pub* __restrict__ pub,
                                               int* __restrict__ seq_ctr, int max_fac, bool publish = true) {
  __shared__ int s_w[17];
  const int nf = m.counters[kCntFactors];
  int status = rc[kRcAbort];
  if (status == 0 && (nf > cap_f || nf > max_fac)) status = kRcBig;
  const int words = (m.counters[kCntNodes] + 31) >> 5;
  const int per = (words + (int)blockDim.x - 1) / (int)blockDim.x;
  const int w0 = threadIdx.x * per, w1 = min(words, w0 + per);
  int cnt = 0;
  for (int w = w0; w < w1; w++) cnt += __popc(bits[w]);
  int total;
  int pos = block_excl_scan(cnt, s_w, &total);
  if (status == 0 && total != nf) status = kRcBig;  // the two counts disagree: let the host path decide
  for (int w = w0; w < w1; w++) {
    uint32_t b = bits[w];
    if (b == 0) continue;
    bits[w] = 0;
    if (status == 0)
      while (b) {
        const int k = __ffs(b) - 1;
        b &= b - 1;
        fac_node[pos++] = (w << 5) + k;
      }
  }
  if (threadIdx.x == 0) {
    const int seq = *seq_ctr + 1;  // the device's count of asynchronous recuts (the host mirrors it)
    *seq_ctr = seq;
    rc[kRcStatus] = status;
    if (publish) {
      pub_store(&pub->rc_status, status);
      pub_store(&pub->rc_nf, nf);
      pub_flag(&pub->seq_rc, seq);
    }
  }
}

// ---- sharded exchange frames packed / checked inside their producer and
// consumer kernels (shard.hip's guard; shard_exchange): one thread closes the
// frame after its payload [0, n - 2) is stored (zeros past the payload are the
// producer's), the consumer tests the summed guard pair against its own x
__device__ __forceinline__ void xchg_close(double* __restrict__ frame, int n, int site, unsigned* __restrict__ seq) {
  const unsigned s = *seq;
  *seq = s + 1;
  const double x = (double)((s & 0xffffu) * 16u + (unsigned)site);
  frame[n - 2] = x;
  frame[n - 1] = x * x;
  frame[n] = x;  // this rank's own x (not exchanged)
}
__device__ __forceinline__ bool xchg_ok(const double* __restrict__ frame, int n, int world) {
  const double x = frame[n];
  return frame[n - 2] == world * x && frame[n - 1] == world * (x * x);
}
// a producer's frame: its consumer checks it (world), reports a mismatch (err, bit 32)
struct XchgArg {
  double* frame;
  unsigned* seq;
  int* err;
  int n, world;
};

}  // namespace vg
