// map.hip — the device-resident adaptive voxel map and the IEKF hot loop.
//
// SURVEY §8(a) rows:
//   A3  var_init / pvec_update           point_utils.cpp:3-65        (fused)
//   A4  cut_voxel_multi -> allocate/push voxel_map.cpp:47-135, octree.cpp:151-228
//   A5  multi_recut -> OctoTree::recut    local_mapping.cpp:144-201, octree.cpp:257-393
//   A6  tras_opt (factor extraction)      octree.cpp:498-521
//   A7  match / OctoTree::match / inside  voxel_map.cpp:241-266, octree.cpp:551-595, 732-737
//   A9  LioStateEstimation point loop     odometry.cpp:111-148
//   A10 multi_margi -> OctoTree::margi    local_mapping.cpp:17-84, octree.cpp:302-333, 395-495
//
// Layout in HBM (vg_internal.h DevMap): a root-voxel open-addressing hash
// (packed 63-bit key -> node id), a node pool of fixed records (NodeHdr 96 B for
// descent, PlaneRec 224 B for the gate, clusters/cov_add/eigen as separate
// arrays), SlideWindow clusters inline per node (W x 80 B), per-physical-slot
// window point arrays (body pnt, world var, owning leaf) and a point_fix arena.
// The reference's pointer-chasing recursion becomes level-synchronous
// worklists; per-leaf accumulation keeps the reference's point order by
// sorting (leaf, order) keys and walking each leaf's segment sequentially, so
// sums are deterministic and order-faithful.
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include "vg_iekf.h"

namespace vg {

// ------------------------------------------------------------------ alloc
int map_alloc(vg_ctx* ctx) {
  DevMap& m = ctx->map;
  const int W = ctx->cfg.win_size;
  m.W = W;
  m.cap_nodes = ctx->cap.max_nodes;
  m.cap_fix = ctx->cap.max_fix_points;
  m.hash_mask = (1 << ctx->cap.hash_log2) - 1;
  m.cap_wp = ctx->cap.max_points_per_scan;
  const size_t cn = m.cap_nodes, hs = (size_t)m.hash_mask + 1, cw = (size_t)m.cap_wp;
  auto ok = [&](void* p) { return p != nullptr; };
  bool good = true;
  good &= ok(m.hdr = ctx->arena.take<NodeHdr>(cn));
  good &= ok(m.pl = ctx->arena.take<PlaneRec>(cn));
  good &= ok(m.pcr_add = ctx->arena.take<Clu>(cn));
  good &= ok(m.pcr_fix = ctx->arena.take<Clu>(cn));
  good &= ok(m.cov_add = ctx->arena.take<double>(cn * kCovN));
  good &= ok(m.eig = ctx->arena.take<double>(cn * 12));
  good &= ok(m.jour = ctx->arena.take<double>(cn));
  good &= ok(m.dbox = ctx->arena.take<double>(cn * 6));
  good &= ok(m.pcrs = ctx->arena.take<Clu>(cn * W));
  good &= ok(m.nscr = ctx->arena.take<int>(cn * 4));
  good &= ok(m.pend = ctx->arena.take<unsigned long long>(cn));
  good &= ok(m.cfirst = ctx->arena.take<int>(cn * 8));
  good &= ok(m.hkey = ctx->arena.take<uint64_t>(hs));
  good &= ok(m.hval = ctx->arena.take<int>(hs));
  good &= ok(m.hfirst = ctx->arena.take<int>(hs));
  good &= ok(m.slide = ctx->arena.take<int>(cn));
  good &= ok(m.in_slide = ctx->arena.take<uint8_t>(cn));
  good &= ok(m.leaf_cnt = ctx->arena.take<int>(cn));
  good &= ok(m.leaf_seg = ctx->arena.take<int>(cn));
  good &= ok(m.fix_pnt = ctx->arena.take<double>((size_t)m.cap_fix * 3));
  good &= ok(m.fix_var = ctx->arena.take<double>((size_t)m.cap_fix * 9));
  good &= ok(m.wp_pnt = ctx->arena.take<double>(cw * W * 3));
  good &= ok(m.wp_var = ctx->arena.take<double>(cw * W * 9));
  good &= ok(m.wp_leaf = ctx->arena.take<int>(cw * W));
  good &= ok(m.wp_int = ctx->arena.take<float>(cw * W));
  m.ord_stride = (int)(cw * (size_t)(ctx->cfg.max_layer + 1));
  good &= ok(m.wp_ord = ctx->arena.take<int>((size_t)m.ord_stride * W));
  good &= ok(m.lseg = ctx->arena.take<uint64_t>(cn * W));
  good &= ok(m.slot_epoch = ctx->arena.take<int>(kMaxWin));
  good &= ok(m.arena = ctx->arena.take<int>(kMaxWin));
  good &= ok(ctx->d_cmap = ctx->arena.take<float4>((cw + 2) / 3));
  good &= ok(ctx->d_cmap_n = ctx->arena.take<int>(4));
  good &= ok(m.counters = ctx->arena.take<int>(kCntN));
  good &= ok(m.stamp = ctx->arena.take<int>(cn));
  good &= ok(m.wpn = ctx->arena.take<int>(kMaxWin));
  Work& w = ctx->wk;
  w.cap = (int)(cw * (W + 1));
  good &= ok(w.k0 = ctx->arena.take<uint64_t>(w.cap));
  good &= ok(w.k1 = ctx->arena.take<uint64_t>(w.cap));
  good &= ok(w.v0 = ctx->arena.take<uint32_t>(w.cap));
  good &= ok(w.v1 = ctx->arena.take<uint32_t>(w.cap));
  good &= ok(w.u0 = ctx->arena.take<uint32_t>(w.cap));
  good &= ok(w.u1 = ctx->arena.take<uint32_t>(w.cap));
  good &= ok(w.ac_cnt = ctx->arena.take<uint32_t>(cn));
  good &= ok(w.ac_off = ctx->arena.take<uint32_t>(cn));
  good &= ok(w.cand = ctx->arena.take<int>(cn));
  good &= ok(w.list0 = ctx->arena.take<int>(cn));
  good &= ok(w.list1 = ctx->arena.take<int>(cn));
  good &= ok(w.list2 = ctx->arena.take<int>(cn));
  good &= ok(w.leaf = ctx->arena.take<int>(cw));
  good &= ok(w.pw = ctx->arena.take<double>(cw * 3));
  good &= ok(w.iekf_cache = ctx->arena.take<int>(cw));
  good &= ok(w.pk_leaf = ctx->arena.take<int>(cw));
  good &= ok(w.rc = ctx->arena.take<int>(128));
  good &= ok(w.cand_bits = ctx->arena.take<uint32_t>(ctx->cap.max_nodes / 32 + 1));
  good &= ok(w.plan = ctx->arena.take<int>(cn * 8));
  w.ngran = (int)(cw / 1024 + 64);
  good &= ok(w.gran = ctx->arena.take<unsigned long long>(w.ngran));
  good &= ok(w.sub_odd = ctx->arena.take<int>(cn));
  good &= ok(w.info_odd = ctx->arena.take<int>(w.cap));
  good &= ok(w.ev_odd = ctx->arena.take<uint64_t>(w.cap));
  w.nparts = 1024;
  good &= ok(w.partials = ctx->arena.take<double>((size_t)w.nparts * 40));
  if (!good) {
    ctx->err = "arena exhausted (map)";
    return VG_E_CAPACITY;
  }
  size_t b1 = 0, b2 = 0;
  VG_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, b1, w.k0, w.k1, w.cap, 0, 64, ctx->stream));
  VG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b2, w.v0, w.v1, w.cap, ctx->stream));
  w.tmp_bytes = (b1 > b2 ? b1 : b2) + 256;
  w.tmp = ctx->arena.take<char>(w.tmp_bytes);
  w.tmp2 = ctx->arena.take<char>(w.tmp_bytes);  // the margi prefix sorts on the second stream
  if (!w.tmp || !w.tmp2) {
    ctx->err = "arena exhausted (sort workspace)";
    return VG_E_CAPACITY;
  }
  return map_set_attrs(ctx);
}

int map_reset(vg_ctx* ctx) {
  DevMap& m = ctx->map;
  hipStream_t s = ctx->stream;
  // Node records are handed out zeroed: the pool is cleared here (all of it
  // the first time, afterwards the ids handed out since), so no allocation on
  // the per-scan path writes a record it has not filled (ids are never reused
  // between resets)
  int used = m.cap_nodes;
  if (ctx->pool_zeroed) {
    VG_HIP(hipMemcpyAsync(ctx->h_pinned, m.counters, kCntN * sizeof(int), hipMemcpyDeviceToHost, s));
    VG_HIP(hipStreamSynchronize(s));
    used = ctx->h_pinned[kCntNodes] < m.cap_nodes ? ctx->h_pinned[kCntNodes] : m.cap_nodes;
  }
  if (used > 0) {
    const size_t u = (size_t)used;
    VG_HIP(hipMemsetAsync(m.pl, 0, u * sizeof(PlaneRec), s));
    VG_HIP(hipMemsetAsync(m.pcr_add, 0, u * sizeof(Clu), s));
    VG_HIP(hipMemsetAsync(m.pcr_fix, 0, u * sizeof(Clu), s));
    VG_HIP(hipMemsetAsync(m.cov_add, 0, u * kCovN * sizeof(double), s));
    VG_HIP(hipMemsetAsync(m.eig, 0, u * 12 * sizeof(double), s));
    VG_HIP(hipMemsetAsync(m.jour, 0, u * sizeof(double), s));
    VG_HIP(hipMemsetAsync(m.pcrs, 0, u * m.W * sizeof(Clu), s));
    VG_HIP(hipMemsetAsync(m.lseg, 0, u * m.W * sizeof(uint64_t), s));
  }
  ctx->pool_zeroed = true;
  const size_t hs = (size_t)m.hash_mask + 1;
  VG_HIP(hipMemsetAsync(m.hkey, 0xff, hs * sizeof(uint64_t), s));
  VG_HIP(hipMemsetAsync(m.hval, 0xff, hs * sizeof(int), s));
  VG_HIP(hipMemsetAsync(m.hfirst, 0x7f, hs * sizeof(int), s));
  VG_HIP(hipMemsetAsync(m.counters, 0, kCntN * sizeof(int), s));
  VG_HIP(hipMemsetAsync(m.stamp, 0, (size_t)m.cap_nodes * sizeof(int), s));
  VG_HIP(hipMemsetAsync(m.wpn, 0, kMaxWin * sizeof(int), s));
  VG_HIP(hipMemsetAsync(m.slot_epoch, 0, kMaxWin * sizeof(int), s));
  VG_HIP(hipMemsetAsync(m.arena, 0, kMaxWin * sizeof(int), s));
  VG_HIP(hipMemsetAsync(ctx->wk.cand_bits, 0, (ctx->cap.max_nodes / 32 + 1) * sizeof(uint32_t), s));
  VG_HIP(hipMemsetAsync(m.in_slide, 0, m.cap_nodes, s));
  VG_HIP(hipMemsetAsync(m.leaf_cnt, 0, (size_t)m.cap_nodes * sizeof(int), s));
  VG_HIP(hipMemsetAsync(m.cfirst, 0x7f, (size_t)m.cap_nodes * 8 * sizeof(int), s));
  VG_HIP(hipMemsetAsync(m.nscr, 0xff, (size_t)m.cap_nodes * 4 * sizeof(int), s));
  VG_HIP(hipStreamSynchronize(s));
  return ds_reset(ctx);  // the pipeline downsample's voxel table
}


// ------------------------------------------------------------------ IEKF
// One IEKF iteration's point loop (odometry.cpp:111-148): world covariance,
// association (cached-leaf fast path or root hash + octree descent), the
// probabilistic point-to-plane gate (octree.cpp:557-579), the Jacobian and the
// weighted normal-equation accumulation. Each block writes 34 partial sums:
// HTH (upper 21), HTz (6), nnt (upper 6), match count (1). fp64 throughout.
__device__ __forceinline__ int descend(const NodeHdr* __restrict__ hdr, int node, const V3& w) {
  for (int d = 0; d < 8 && node >= 0; d++) {
    const NodeHdr& h = hdr[node];
    if (h.octo == 0) return node;
    node = h.child[octant(w, h.center)];
  }
  return -1;
}

// OctoTree::match at a leaf; returns 1 and sigma on success
__device__ __forceinline__ int match_leaf(const NodeHdr& h, const PlaneRec& P, const V3& wld, const M3& var_wld,
                                          double& sigma) {
  if (!h.is_plane) return 0;
  V3 c = ld_v3(P.center), n = ld_v3(P.normal);
  V3 d = sub(wld, c);
  float dis_to_plane = fabs(dot3(n, d));
  V3 cw = sub(c, wld);
  float dis_to_center = cw[0] * cw[0] + cw[1] * cw[1] + cw[2] * cw[2];
  float range_dis = (dis_to_center - dis_to_plane * dis_to_plane);
  if (!(range_dis <= 3 * 3 * P.radius)) return 0;
  double J[6] = {d[0], d[1], d[2], -n[0], -n[1], -n[2]};
  double t[6];
  for (int j = 0; j < 6; j++) {
    double s = J[0] * P.var[sym_idx(6, 0, j)];
    for (int k = 1; k < 6; k++) s += J[k] * P.var[sym_idx(6, k, j)];
    t[j] = s;
  }
  double sl = t[0] * J[0];
  for (int j = 1; j < 6; j++) sl += t[j] * J[j];
  V3 vn = mul(var_wld, n);
  sl += dot3(n, vn);
  if (dis_to_plane < 3 * sqrt(sl)) {
    sigma = sl;
    return 1;
  }
  return 0;
}

__device__ __forceinline__ bool inside(const NodeHdr& h, const V3& w) {
  double hl = h.qlen * 2;
  return (w[0] >= h.center[0] - hl && w[0] <= h.center[0] + hl && w[1] >= h.center[1] - hl &&
          w[1] <= h.center[1] + hl && w[2] >= h.center[2] - hl && w[2] <= h.center[2] + hl);
}


// ---- wave sums without LDS: the partner across lane bit L (lane ^ L) via
// gfx950's v_permlane32_swap / v_permlane16_swap and DPP (row_ror:8, row
// shifts by 4, quad perms)
__device__ __forceinline__ double pack_d(unsigned lo, unsigned hi) {
  return __longlong_as_double(((long long)hi << 32) | lo);
}
template <int C>
__device__ __forceinline__ unsigned dpp32(unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, C, 0xf, 0xf, false);
}
template <int L>
__device__ __forceinline__ double xor_lane(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
  if constexpr (L == 32) {  // r[0] = x[lane % 32], r[1] = x[lane % 32 + 32]
    auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return (lane & 32) ? pack_d(l2[0], h2[0]) : pack_d(l2[1], h2[1]);
  } else if constexpr (L == 16) {  // r[0] = the even row's x, r[1] = the odd row's
    auto l2 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto h2 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return (lane & 16) ? pack_d(l2[0], h2[0]) : pack_d(l2[1], h2[1]);
  } else if constexpr (L == 8) {
    return pack_d(dpp32<0x128>(lo), dpp32<0x128>(hi));  // row_ror:8
  } else if constexpr (L == 4) {
    const double up = pack_d(dpp32<0x104>(lo), dpp32<0x104>(hi));  // row_shl:4 (lane i <- i + 4)
    const double dn = pack_d(dpp32<0x114>(lo), dpp32<0x114>(hi));  // row_shr:4 (lane i <- i - 4)
    return (lane & 4) ? dn : up;
  } else if constexpr (L == 2) {
    return pack_d(dpp32<0x4E>(lo), dpp32<0x4E>(hi));  // quad_perm [2,3,0,1]
  } else {
    return pack_d(dpp32<0xB1>(lo), dpp32<0xB1>(hi));  // quad_perm [1,0,3,2]
  }
}
// one level of a halving wave sum: the lanes with bit L clear keep the first
// ceil(N/2) values, the others the rest, each adding its partner's copy
template <int L, int N>
__device__ __forceinline__ void halve(const double (&v)[N], double (&w)[(N + 1) / 2], int lane, int& idx, int& n) {
  constexpr int H = (N + 1) / 2;
  const bool hi = (lane & L) != 0;
#pragma unroll
  for (int j = 0; j < H; j++) {
    const double a = v[j], b = (H + j < N) ? v[H + j] : 0.0;
    w[j] = (hi ? b : a) + xor_lane<L>(hi ? a : b, lane);
  }
  if (hi) {
    idx += H;
    n = n > H ? n - H : 0;
  } else {
    n = n < H ? n : H;
  }
}

// The pose (x_curr R, p and the rotation / translation covariance blocks) is
// read from the device state the previous k_iekf_update wrote; the kernel is a
// no-op once the IEKF has finished (st->done). Iteration 0 ignores the leaf
// cache (no association yet, odometry.cpp:111-132).
// one IEKF iteration's point loop over the workgroup's chunk vb (k_iekf): the
// 34 sums of this lane's points
// kPf: a point whose cached leaf matched last iteration (octos[i]) touches its
// plane record's 128 B lines right away, beside the header load, so the
// gate's record reads hit in cache instead of a second dependent miss
template <bool kPf = false>
__device__ __forceinline__ void iekf_points(const MP& mp, const DState* __restrict__ st, const DevMap& m,
                                            int* __restrict__ cache, int* __restrict__ pk, int it, int nb, int vb,
                                            const M3& R, const V3& p, const M3& rot_var, const M3& tsl_var,
                                            double (&acc)[kIekfVals]) {
  const int* __restrict__ keep = iekf_keep(st);
  const int n = keep ? st->snk : st->sn;
  const float* __restrict__ x = st->sx;
  const float* __restrict__ y = st->sy;
  const float* __restrict__ z = st->sz;
  const M3 Rt = tr(R);
  for (int j = 0; j < kIekfVals; j++) acc[j] = 0.0;
  for (int q = vb * blockDim.x + threadIdx.x; q < n; q += nb * blockDim.x) {
    const int i = keep ? keep[q] : q;  // the raw index (the memo and the profiling pass are per raw point)
    V3 pnt;
    M3 var;
    var_init_pt(mp, x[i], y[i], z[i], pnt, var);
    M3 var_world = world_var(R, var, pnt, rot_var, tsl_var);
    V3 wld = rigid(R, pnt, p);
    // cache[i]: the leaf of the point's last match (the reference's octos[i],
    // odometry.cpp:124-131, reset per scan) or, after a failed match, the
    // leaf the descent reached — a memo only (bit 30 tags it): while the
    // point stays inside that leaf's box and its float voxel key still names
    // the leaf's root (the lookup rounds in float, voxel_map.cpp:246-253), the
    // lookup would reach the same leaf, so unmatched points skip the hash +
    // descent too
    const int cv = it > 0 ? cache[i] : -1;
    int leaf = cv >= 0 ? (cv & 0x3fffffff) : -1;
    int flag = 0;
    double sigma = 0;
    double pf0 = 0.0, pf1 = 0.0, pf2 = 0.0;
    if (kPf && cv >= 0 && !(cv & 0x40000000)) {  // bytes 0, 112, 216: every 128 B line the 224 B record spans
      const double* rec = reinterpret_cast<const double*>(&m.pl[leaf]);
      pf0 = rec[0];
      pf1 = rec[14];
      pf2 = rec[27];
    }
    // a matched leaf (octos[i]): OctoTree::inside's inclusive box; a memo: the
    // descent's own region (dbox: strict where the descent is strict), so a
    // point on a centre plane is never kept in the wrong sibling
    bool hit = leaf >= 0 && ((cv & 0x40000000) ? in_dbox(m.dbox + (size_t)leaf * 6, wld) : inside(m.hdr[leaf], wld));
    if (hit && (cv & 0x40000000)) {
      uint64_t kw, kl;
      const NodeHdr& hl = m.hdr[leaf];
      hit = pack_key(wld, mp.vs, kw) && pack_key(v3(hl.center[0], hl.center[1], hl.center[2]), mp.vs, kl) && kw == kl;
    }
    if (hit) {
      if (kPf) asm volatile("" ::"v"(pf0), "v"(pf1), "v"(pf2));  // the touches complete here, not before
      flag = match_leaf(m.hdr[leaf], m.pl[leaf], wld, var_world, sigma);
      if (!flag && !(cv & 0x40000000)) leaf = -2;  // the reference's octos[i] stays: keep the cache
    } else {
      leaf = -1;
      uint64_t key;
      if (pack_key(wld, mp.vs, key) && owns(m, key)) {  // another shard's tile: not matched here
        int root = hash_find(m.hkey, m.hval, m.hash_mask, key);
        int lf = root >= 0 ? descend(m.hdr, root, wld) : -1;
        if (lf >= 0) {
          flag = match_leaf(m.hdr[lf], m.pl[lf], wld, var_world, sigma);
          leaf = lf;
        }
      }
    }
    if (pk) pk[i] = flag ? leaf : -1;  // the leaf whose plane this iteration read (profiling pass)
    if (flag) {
      cache[i] = leaf;
    } else if (leaf >= 0) {
      if (it == 0 || cv < 0 || (cv & 0x40000000)) cache[i] = leaf | 0x40000000;  // no octos[i] to keep
    } else if (leaf == -1 && (it == 0 || cv < 0 || (cv & 0x40000000))) {
      cache[i] = -1;
    }
    if (flag) {
      const PlaneRec& P = m.pl[leaf];
      V3 nn = ld_v3(P.normal), c = ld_v3(P.center);
      double R_inv = 1.0 / (0.0005 + sigma);
      double resi = dot3(nn, sub(wld, c));
      V3 j3 = mul(mul(hat(pnt), Rt), nn);
      double jac[6] = {j3[0], j3[1], j3[2], nn[0], nn[1], nn[2]};
      int k = 0;
      for (int r = 0; r < 6; r++) {
        double jr_ = jac[r] * R_inv;
        for (int c2 = r; c2 < 6; c2++, k++) acc[k] += jr_ * jac[c2];
      }
      for (int r = 0; r < 6; r++) acc[21 + r] -= jac[r] * (R_inv * resi);
      acc[27] += nn[0] * nn[0];
      acc[28] += nn[0] * nn[1];
      acc[29] += nn[0] * nn[2];
      acc[30] += nn[1] * nn[1];
      acc[31] += nn[1] * nn[2];
      acc[32] += nn[2] * nn[2];
      acc[33] += 1.0;
    }
  }
}
// the workgroup's 34 sums (threads < 34 hold one each): a halving butterfly
// per wave, then LDS across the 4 waves (fixed tree). Every level pairs lane ^
// L for L = 32, 16, ..., 1, so each sum is bit for bit lane 0's of a shfl_down
// tree, but a lane hands over half of the values it carries at every level:
// 37 exchanges for the 34 sums instead of 204, through permlane / DPP
__device__ __forceinline__ double iekf_wg_sum(double (&acc)[kIekfVals], double (*red)[kIekfVals]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  static_assert(kIekfVals == 34, "the halving levels below are laid out for 34 sums");
  int ridx = 0, rn = kIekfVals;
  double h17[17], h9[9], h5[5], h3[3], h2[2], h1[1];
  halve<32>(acc, h17, lane, ridx, rn);
  halve<16>(h17, h9, lane, ridx, rn);
  halve<8>(h9, h5, lane, ridx, rn);
  halve<4>(h5, h3, lane, ridx, rn);
  halve<2>(h3, h2, lane, ridx, rn);
  halve<1>(h2, h1, lane, ridx, rn);
  if (rn == 1) red[wv][ridx] = h1[0];
  __syncthreads();
  const int j = threadIdx.x < kIekfVals ? threadIdx.x : 0;
  return ((red[0][j] + red[1][j]) + red[2][j]) + red[3][j];
}
// the pose words an iteration's point loop reads from x_curr: R 9, p 3, the
// rotation and translation covariance blocks 9 + 9
__device__ __forceinline__ double pose_word(const double* xc, int t) {
  if (t < 12) return xc[t];
  if (t < 21) return xc[kXS + ((t - 12) / 3) * 15 + (t - 12) % 3];
  return xc[kXS + (3 + (t - 21) / 3) * 15 + 3 + (t - 21) % 3];
}
__device__ __forceinline__ void pose_of(const double* w, M3& R, V3& p, M3& rot_var, M3& tsl_var) {
  for (int q = 0; q < 9; q++) {
    R[q] = w[q];
    rot_var[q] = w[12 + q];
    tsl_var[q] = w[21 + q];
  }
  p = v3(w[9], w[10], w[11]);
}

template <bool kPf>
__global__ void __launch_bounds__(256) k_iekf(MP mp, DState* __restrict__ st, int it, DevMap m,
                                              int* __restrict__ cache, double* __restrict__ partials,
                                              int* __restrict__ pk) {
  if (st->done) return;
  // the scan's critical chain: its waves issue ahead of co-resident waves of
  // the previous scan's margi remainder (k_margi_copy) on a shared SIMD
  __builtin_amdgcn_s_setprio(2);
  const bool clk_on = st->clk.on != 0;
  const int clk_slot = (st->clk.scan * 4 + it) & (kClkRing - 1);
  if (clk_on && blockIdx.x == 0 && threadIdx.x == 0) {
    st->clk.t0[clk_slot] = (unsigned long long)wall_clock64();
    st->clk.exec[clk_slot] = 1;
  }
  VG_PROBE_BEGIN();
  const int n = st->sn;
  double w[30];
  for (int t = 0; t < 30; t++) w[t] = pose_word(st->xc, t);
  M3 R, rot_var, tsl_var;
  V3 p;
  pose_of(w, R, p, rot_var, tsl_var);
  // XCD-aware chunking (cdna_hip_programming.md T1): blocks are dealt
  // round-robin over the 8 XCDs, so block b works on chunk (b % 8) * (nb / 8)
  // + b / 8 — each XCD sweeps a contiguous run of the scan and the plane /
  // node records of neighbouring points stay in its own L2 (nb % 8 == 0)
  const int nb = gridDim.x;
  const int vb = iekf_chunk(blockIdx.x, nb);
  double acc[kIekfVals];
  iekf_points<kPf>(mp, st, m, cache, pk, it, nb, vb, R, p, rot_var, tsl_var, acc);
  if (blockIdx.x == 0 && threadIdx.x == 0) st->iekf_pts += iekf_n(st);  // (vg_stats::iekf_points)
  if (blockIdx.x == 0) VG_PROBE_MARK(30);  // the point loop (thread 0 of block 0)
  __shared__ double red[4][kIekfVals];
  const double v = iekf_wg_sum(acc, red);
  if (threadIdx.x < kIekfVals) partials[(size_t)blockIdx.x * kIekfVals + threadIdx.x] = v;
  if (clk_on && blockIdx.x < kClkBlocks) {  // the workgroup's end (its partials written)
    __syncthreads();
    if (threadIdx.x == 0) st->clk.tend[clk_slot][blockIdx.x] = (unsigned long long)wall_clock64();
  }
  if (blockIdx.x == 0) VG_PROBE_MARK(31);  // the block reduction
#ifdef VG_PROBE
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_probe[59], 1ull);
#endif
}

// the IEKF's end to the insert's stream (vg_ctx::d_sync[1]): every thread's
// state writes released at agent scope (one workgroup: one L2 write-back),
// then the flag advances by one
__device__ __forceinline__ void iekf_signal_done(unsigned* flag) {
  if (!flag) return;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// P_k of SURVEY 8(d), the profiling pass only: distinct plane records the
// iteration read, deduplicated with a per-node tag (outside k_iekf's timing)
__global__ void __launch_bounds__(256) k_iekf_planes(const DState* __restrict__ st, DevMap m,
                                                     const int* __restrict__ pk, int tag, int* __restrict__ out) {
  if (st->done) return;
  const int* keep = iekf_keep(st);
  const int n = iekf_n(st);
  int cnt = 0;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const int leaf = pk[keep ? keep[q] : q];
    if (leaf >= 0 && m.stamp[leaf] != tag && atomicExch(&m.stamp[leaf], tag) != tag) cnt++;
  }
  wave_append(out, cnt);
}

// The IEKF update of iteration `it` (vg_iekf.h) as its own one-workgroup
// launch. (A last-workgroup-done ticket inside k_iekf would need an
// agent-scope release per workgroup, which on the multi-XCD MI355X writes back
// the XCD's L2 each time: measured ~20 us per iteration, far more than the
// launch it saves.)
// done_flag: the update that finishes the IEKF also advances the IEKF ->
// insert hand-off flag (one workgroup: one release), so no k_sync_set launch
// follows the IEKF graph
__global__ void __launch_bounds__(1024) k_iekf_update(int nb, const double* __restrict__ partials,
                                                     DState* __restrict__ st, int it, unsigned* done_flag,
                                                     int xworld, int* xerr) {
  __shared__ IekfLds L;
  if (st->done) return;
  __builtin_amdgcn_s_setprio(2);  // (k_iekf)
  iekf_update_block(nb, partials, st, it, L, xworld, xerr);
  if (done_flag && L.fin) iekf_signal_done(done_flag);
}
// sharded mode: this shard's 34 sums (the update then runs on the all-reduced ones)
// sharded mode: this shard's 34 sums, packed into the exchange frame (the
// update runs on the all-reduced frame, k_iekf_update checks its guard); an
// iteration after convergence still closes the frame (the exchange runs)
__global__ void __launch_bounds__(1024) k_iekf_reduce(int nb, const double* __restrict__ partials,
                                                     const DState* __restrict__ st, XchgArg xa) {
  __shared__ IekfLds L;
  const bool done = st->done;
  if (!done) {
    const int n = iekf_n(st);
    iekf_reduce_block(nb, partials, L, n < nb * 256 ? (n + 255) / 256 : nb);
  }
  for (int i = threadIdx.x; i < xa.n - 2; i += blockDim.x) xa.frame[i] = (!done && i < kIekfVals) ? L.o[i] : 0.0;
  if (threadIdx.x == 0) xchg_close(xa.frame, xa.n, 0, xa.seq);
}

// grid of the IEKF point loop: sized by the context's capacity (the kernels
// read the scan size from the device state), a multiple of the 8 XCDs
static int iekf_blocks(vg_ctx* ctx) {
  return ((grid_for(ctx->cap.max_points_per_scan, 256, 512) + 7) / 8) * 8;
}
int iekf_grid(vg_ctx* ctx) { return iekf_blocks(ctx); }

// one IEKF iteration: the point loop (block partials) and the update; the
// optional event pair brackets k_iekf alone (vg_profile)
int iekf_iteration(vg_ctx* ctx, const MP& mp, const float* x, const float* y, const float* z, int n, int it,
                   hipEvent_t ev0, hipEvent_t ev1, int tag, hipStream_t s, unsigned* done_flag) {
  Work& w = ctx->wk;
  if (!s) s = ctx->stream;
  (void)x;
  (void)y;
  (void)z;
  (void)n;  // the scan is read from the device state (state_set_scan)
  const int nb = iekf_blocks(ctx);
  if (ev0) VG_HIP(hipEventRecord(ev0, s));
  auto kern = ctx->iekf_prefetch ? k_iekf<true> : k_iekf<false>;
  kern<<<nb, 256, 0, s>>>(mp, ctx->st, it, ctx->map, w.iekf_cache, w.partials, tag ? w.pk_leaf : nullptr);
  if (ev1) VG_HIP(hipEventRecord(ev1, s));
  if (tag) k_iekf_planes<<<nb, 256, 0, s>>>(ctx->st, ctx->map, w.pk_leaf, tag, &ctx->st->planes[it]);
  if (sharded(ctx)) {  // this shard's sums packed into the frame, all-reduced, then the (replicated) update
    Shard& sh = ctx->shard;
    const XchgArg xa{sh.d_frame, sh.d_seq, ctx->map.counters + kCntErr, kShardSmall, sh.world};
    k_iekf_reduce<<<1, 1024, 0, s>>>(nb, w.partials, ctx->st, xa);  // (the unsharded update's 60 row groups)
    VG_TRY(shard_exchange(ctx, kShardSmall, s));
    k_iekf_update<<<1, 1024, 0, s>>>(-1, sh.d_frame, ctx->st, it, nullptr, sh.world, ctx->map.counters + kCntErr);
  } else {
    k_iekf_update<<<1, 1024, 0, s>>>(nb, w.partials, ctx->st, it, done_flag, 0, nullptr);
  }
  VG_HIP(hipGetLastError());
  return VG_OK;
}

// ---- sharded mode (world > 1): the scan's points this rank can match ----
// A point is matched only in its own root voxel (A7, voxel_map.cpp:241-266),
// and only the owner of the voxel's tile holds it. At the
// scan's opening pose each raw point's world position w is taken with a box of
// kKeepM metres around it; the key rule is monotone in each coordinate, so
// the voxel keys of the box are those between the keys of w - kKeepM and
// w + kKeepM, and the point is kept when a tile of those keys is this rank's:
// one pass and a prefix sum per scan, and the IEKF's four iterations then
// transform and test only those (DState::skeep). The list holds while every
// point moved less than kmargin = kKeepM since the opening (iekf_keep, checked
// per iteration on the device), else the iteration takes every point. owns()
// still decides per point and iteration, so the matches are the unsharded
// path's either way; only the order of the fp sums within a rank follows the
// list.
constexpr double kKeepM = 0.1;
__global__ void __launch_bounds__(256) k_keep_flags(MP mp, const DState* __restrict__ st, DevMap m,
                                                    int* __restrict__ flag, unsigned* __restrict__ rmax_bits) {
  const int n = st->sn;
  const float* __restrict__ x = st->sx;
  const float* __restrict__ y = st->sy;
  const float* __restrict__ z = st->sz;
  M3 R;
  for (int q = 0; q < 9; q++) R[q] = st->xc[q];
  const V3 p = v3(st->xc[9], st->xc[10], st->xc[11]);
  const M3 eR = ld_m3(mp.extR);
  const V3 et = ld_v3(mp.extt);
  float rmax = 0.0f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const V3 pnt = rigid(eR, v3(x[i], y[i], z[i]), et);
    const V3 w = rigid(R, pnt, p);
    rmax = fmaxf(rmax, (float)norm3(pnt));
    int64_t lo[3], hi[3];
    bool in = true;
    for (int j = 0; j < 3; j++) {
      const int64_t k0 = key_axis_d(w[j] - kKeepM, mp.vs) + kKeyOff, k1 = key_axis_d(w[j] + kKeepM, mp.vs) + kKeyOff;
      lo[j] = (k0 > 0 ? k0 : 0) >> 4;  // (keys outside the packed range are never matched)
      hi[j] = (k1 < 2 * kKeyOff - 1 ? k1 : 2 * kKeyOff - 1) >> 4;
      in &= k1 >= 0 && k0 < 2 * kKeyOff;
    }
    int keep = 0;
    if (in)
      for (int64_t tx = lo[0]; tx <= hi[0] && !keep; tx++)
        for (int64_t ty = lo[1]; ty <= hi[1] && !keep; ty++)
          for (int64_t tz = lo[2]; tz <= hi[2] && !keep; tz++)
            keep = tile_owner_t((uint64_t)tx, (uint64_t)ty, (uint64_t)tz, m.shard_world) == m.shard_rank;
    flag[i] = keep;
  }
  for (int off = 32; off > 0; off >>= 1) rmax = fmaxf(rmax, __shfl_down(rmax, off, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(rmax_bits, __float_as_uint(rmax));  // (non-negative: ordered as bits)
}
__global__ void __launch_bounds__(256) k_keep_scatter(MP mp, DState* __restrict__ st, const int* __restrict__ flag,
                                                      const int* __restrict__ pos, int* __restrict__ list,
                                                      const unsigned* __restrict__ rmax_bits) {
  const int n = st->sn;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    if (flag[i]) list[pos[i]] = i;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->snk = n > 0 ? pos[n - 1] + flag[n - 1] : 0;
    st->skeep = list;
    for (int t = 0; t < 12; t++) st->kpose[t] = st->xc[t];
    st->krmax = (double)__uint_as_float(*rmax_bits) * (1.0 + 1e-6) + 1e-6;  // (the float max rounded up)
    st->kmargin = kKeepM;
  }
}
static int keep_list(vg_ctx* ctx, const MP& mp, int n, hipStream_t s) {
  Shard& sh = ctx->shard;
  if (n <= 0) n = 1;  // (an empty scan: the kernels read the count from the state)
  VG_HIP(hipMemsetAsync(sh.keep_rmax, 0, sizeof(unsigned), s));
  const int g = grid_for(n);
  k_keep_flags<<<g, kBlock, 0, s>>>(mp, ctx->st, ctx->map, sh.keep_flag, sh.keep_rmax);
  size_t tb = sh.keep_tmp_bytes;
  VG_HIP(hipcub::DeviceScan::ExclusiveSum(sh.keep_tmp, tb, sh.keep_flag, sh.keep_pos, n, s));
  k_keep_scatter<<<g, kBlock, 0, s>>>(mp, ctx->st, sh.keep_flag, sh.keep_pos, sh.keep_list, sh.keep_rmax);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

// the four IEKF iterations (odometry.cpp:68). The launches do not change from
// scan to scan, so an unsharded context captures them once and replays the
// graph: one host call instead of eight launches, and the device starts each
// node without the per-launch dispatch gap. The per-stage profiling pass
// (vg_profile bit 1) launches directly, with an event pair around each k_iekf.
int iekf_run(vg_ctx* ctx, const MP& mp, const float* x, const float* y, const float* z, int n, int bank,
             const double* begin_xc, hipStream_t s, const PropArg* begin_prop, bool signal, bool* signalled,
             bool opened) {
  if (!s) s = ctx->stream;
  if (signalled) *signalled = false;
  if (begin_xc || begin_prop)  // the scan opens here (pipeline.cpp)
    VG_TRY(state_scan_begin(ctx, begin_xc, x, y, z, n, s, begin_prop));
  else if (!opened) VG_TRY(state_set_scan(ctx, x, y, z, n, s));
  if (sharded(ctx) && ctx->shard.world > 1) VG_TRY(keep_list(ctx, mp, n, s));  // at the opening pose
  const bool graph = ctx->use_graphs && !sharded(ctx) && !ctx->prof_stages;
  const bool ev = ctx->prof_on && !graph;
  // the last update signals the hand-off itself (k_iekf_update; not when sharded)
  const bool self_signal = signal && !sharded(ctx);
  unsigned* flag = self_signal ? ctx->d_sync + 1 : nullptr;
  auto enqueue = [&]() -> int {
    for (int it = 0; it < 4; it++)
      VG_TRY(iekf_iteration(ctx, mp, x, y, z, n, it, ev ? ctx->iekf_ev[bank + it][0] : nullptr,
                            ev ? ctx->iekf_ev[bank + it][1] : nullptr,
                            graph || !ctx->prof_stages ? 0 : ++ctx->plane_tag, s, flag));
    return VG_OK;
  };
  if (!graph) {
    VG_TRY(enqueue());
    if (signalled) *signalled = self_signal;
    return VG_OK;
  }
  hipGraphExec_t& ge = ctx->g_iekf[self_signal ? 3 : 0];
  if (!ge) {
    std::lock_guard<std::recursive_mutex> cap_lk_(capture_mutex());  // (vg_internal.h)
    VG_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    const int r = enqueue();
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(s, &g);
    if (r != VG_OK) return r;
    VG_HIP(e);
    VG_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    VG_HIP(hipGraphDestroy(g));
  }
  VG_HIP(hipGraphLaunch(ge, s));
  if (signalled) *signalled = self_signal;
  return VG_OK;
}

// ------------------------------------------------------------------ insert (A3/A4)
// per downsampled point: var_init + pvec_update (world var), world point, root
// key insert-or-find, first-occurrence marking of brand-new keys.
// kPre (the initialisation's cut_voxel, initialization.cpp:229-246): body
// points already motion-compensated (pin, fp64), the pose and covariance of
// x_buf[i] in xsrc (kXC layout), and either the identity body covariance
// without pvec_update (var_identity, rounds before convergence) or calcBodyVar
// on the body point + pvec_update.
template <bool kPre>
__global__ void __launch_bounds__(256) k_ins_prep(int n_arg, const int* __restrict__ nd, const float* __restrict__ ox, const float* __restrict__ oy,
                           const float* __restrict__ oz, const float* __restrict__ oi, MP mp, DState* __restrict__ st, int slot,
                           DevMap m, double* __restrict__ pw, uint32_t* __restrict__ hslot,
                           const PushArg* __restrict__ pa, const double* __restrict__ pin, const double* __restrict__ xsrc,
                           int var_identity, int* __restrict__ dsf, unsigned long long* __restrict__ gran, int ngran,
                           const int* __restrict__ ph_in) {
  const int n = nd ? *nd : n_arg;  // the downsampled count on the device (ds_enqueue_hashed)
  {  // the root registration's look-back granules (k_ins_roots_lb, the next launch) start empty
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (gran && g < ngran) gran[g] = 0ull;
  }
  // the window push (local_mapping.cpp:434-441) rides in block 0: it copies
  // x_curr into x_buf[ord], which this kernel only reads
  if (!kPre && pa && blockIdx.x == 0) push_state_block(st, *pa);  // pa: host-mapped (vg_ctx::d_in)
  // the scan graph's per-scan numbers (HostIn::ph, host-mapped) into the device state, beside the push
  if (ph_in && blockIdx.x == 0 && threadIdx.x < 6) st->ph[threadIdx.x] = ph_in[threadIdx.x];
  // pose of x_buf[ord] = x_curr after the IEKF (device state)
  const double* xc = kPre ? xsrc : st->xc;
  M3 R, rot_var, tsl_var;
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      R(r, c) = xc[r * 3 + c];
      rot_var(r, c) = xc[kXS + r * 15 + c];
      tsl_var(r, c) = xc[kXS + (3 + r) * 15 + 3 + c];
    }
  const V3 p = ld_v3(xc + 9);
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // per-insert device counters (read by the later kernels)
    m.counters[kCntNew] = m.counters[kCntNodes];  // first id of this scan's new roots
    m.counters[kCntSlideBase] = m.counters[kCntSlide];  // surf_map_slide size before this scan's roots
    m.counters[kCntTouched] = 0;
    m.counters[kCntCreate] = 0;
    m.counters[kCntSeg] = 0;
    m.counters[kCntMisc] = 0;  // insert abort flag (child-allocation overflow)
    m.counters[kCntPlaneUpd] = 0;  // margi's per-scan branch counters (vg_stats)
    m.counters[kCntFixFull] = 0;
    m.counters[kCntNds] = n;
    m.wpn[slot] = n;  // window points of this physical slot (k_make_win)
    m.slot_epoch[slot] += 1;  // every leaf run of the slot's previous scan is stale now
    m.arena[slot] = m.cap_wp;
    if (dsf && dsf[0]) {  // the downsample's key-range error (no host wait in between)
      atomicOr(&m.counters[kCntErr], 1);
      dsf[0] = 0;
    }
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    V3 pnt;
    M3 vw;
    if (kPre) {
      pnt = v3(pin[(size_t)i * 3], pin[(size_t)i * 3 + 1], pin[(size_t)i * 3 + 2]);
      if (var_identity) {
        vw = M3::I();
      } else {
        const M3 var = calc_body_var(pnt, mp.dept, mp.beam_dv);
        vw = world_var(R, var, pnt, rot_var, tsl_var);
      }
    } else {
      M3 var;
      var_init_pt(mp, ox[i], oy[i], oz[i], pnt, var);
      vw = world_var(R, var, pnt, rot_var, tsl_var);
    }
    V3 w = rigid(R, pnt, p);
    size_t base = (size_t)slot * m.cap_wp + i;
    for (int j = 0; j < 3; j++) m.wp_pnt[base * 3 + j] = pnt[j];
    for (int j = 0; j < 9; j++) m.wp_var[base * 9 + j] = vw[j];
    m.wp_leaf[base] = -1;
    m.wp_int[base] = oi ? oi[i] : 0.f;
    for (int j = 0; j < 3; j++) pw[(size_t)i * 3 + j] = w[j];
    uint64_t key;
    if (!pack_key(w, mp.vs, key)) {
      atomicOr(&m.counters[kCntErr], 1);
      hslot[i] = 0xffffffffu;
      continue;
    }
    if (!owns(m, key)) {  // another shard's tile (sharded mode)
      hslot[i] = 0xffffffffu;
      continue;
    }
    bool fresh;
    int s = hash_insert(m.hkey, m.hash_mask, key, fresh);
    if (s < 0) {
      atomicOr(&m.counters[kCntErr], 2);
      hslot[i] = 0xffffffffu;
      continue;
    }
    hslot[i] = (uint32_t)s;
    atomicMin(&m.hfirst[s], i);  // the root's first point this scan (k_ins_flags)
  }
}

__global__ void __launch_bounds__(256) k_ins_newflag(int n, const uint32_t* __restrict__ hslot, const int* __restrict__ hval,
                              const int* __restrict__ hfirst, uint32_t* __restrict__ flag) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    uint32_t s = hslot[i];
    flag[i] = (s != 0xffffffffu && hval[s] < 0 && hfirst[s] == i) ? 1u : 0u;
  }
}

// Root registration of cut_voxel_multi (voxel_map.cpp:57-90) in two launches
// (flags + per-tile ranks, then allocation), replacing a flag / scan /
// allocate / count / zero / touch chain. Points are taken in index tiles of
// kRootTile; a point is its root's first point this scan iff hfirst[slot] == i
// (k_ins_prep). Per tile: how many first points, new roots, and roots joining
// surf_map_slide (new ones, and existing ones not yet in it), with each
// point's rank inside its tile. Ids and slide positions then follow point
// index order: deterministic.
constexpr int kRootTile = 1024;  // points per workgroup (256 threads x 4)
__device__ __forceinline__ int ins_root_code(const DevMap& m, const uint32_t* __restrict__ hslot, int i, int n) {
  // bit 0: first point of its root, bit 1: new root, bit 2: joins the slide map
  if (i >= n) return 0;
  const uint32_t s = hslot[i];
  if (s == 0xffffffffu || m.hfirst[s] != i) return 0;
  const int r = m.hval[s];
  if (r < 0) return 7;
  return m.in_slide[r] ? 1 : 5;
}
// exclusive block scan of three counts packed 3 x 21 bits
typedef unsigned long long u64;
__device__ __forceinline__ u64 pack3(int code) {
  return (u64)(code & 1) | ((u64)((code >> 1) & 1) << 21) | ((u64)((code >> 2) & 1) << 42);
}
__device__ __forceinline__ u64 block_excl_scan3(u64 v, u64* s_w, u64* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  u64 x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const u64 y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  u64 base = 0, tot = 0;
  for (int k = 0; k < nw; k++) {
    if (k < wv) base += s_w[k];
    tot += s_w[k];
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}
__global__ void __launch_bounds__(256) k_ins_flags(int n_arg, const int* __restrict__ nd, const uint32_t* __restrict__ hslot, DevMap m,
                                                   uint32_t* __restrict__ rank, int* __restrict__ tile_cnt) {
  const int n = nd ? *nd : n_arg;  // the downsampled count on the device (ds_enqueue_hashed)
  __shared__ u64 s_w[4];
  const int i0 = blockIdx.x * kRootTile + threadIdx.x * 4;
  int code[4];
  u64 v = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    code[k] = ins_root_code(m, hslot, i0 + k, n);
    v += pack3(code[k]);
  }
  u64 tot;
  u64 r = block_excl_scan3(v, s_w, &tot);
  constexpr u64 kF = (1ull << 21) - 1;
#pragma unroll
  for (int k = 0; k < 4; k++) {  // rank: new-root rank | slide rank << 16 (< 1024 each), code in the top bits
    if (i0 + k < n)
      rank[i0 + k] = (unsigned)((r >> 21) & kF) | ((unsigned)((r >> 42) & kF) << 16) | ((unsigned)code[k] << 29);
    r += pack3(code[k]);
  }
  if (threadIdx.x == 0) {
    tile_cnt[blockIdx.x * 3 + 0] = (int)(tot & kF);
    tile_cnt[blockIdx.x * 3 + 1] = (int)((tot >> 21) & kF);
    tile_cnt[blockIdx.x * 3 + 2] = (int)((tot >> 42) & kF);
  }
}
// new roots at kCntNew + (new roots of earlier tiles) + rank, centre
// (0.5 + k) voxel_size, records zeroed; existing first-touched roots isexist
// (voxel_map.cpp:70); slide appends in point order; the root counters. The
// point -> root lookup itself is left to k_ins_descend (after this launch).
__global__ void __launch_bounds__(256) k_ins_roots_alloc(int n_arg, const int* __restrict__ nd, int ntile, const uint32_t* __restrict__ hslot,
                                                         const uint32_t* __restrict__ rank,
                                                         const int* __restrict__ tile_cnt, MP mp, DevMap m) {
  const int n = nd ? *nd : n_arg;  // the downsampled count on the device (ds_enqueue_hashed)
  __shared__ int s_red[3][4];
  int a[3] = {0, 0, 0}, t[3] = {0, 0, 0};
  for (int b = threadIdx.x; b < ntile; b += blockDim.x)
    for (int j = 0; j < 3; j++) {
      const int c = tile_cnt[b * 3 + j];
      t[j] += c;
      if (b < (int)blockIdx.x) a[j] += c;
    }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int off[3], tot[3];
  for (int j = 0; j < 3; j++) {  // (a: this tile's offset, t: the totals) over the block
    int x = a[j], y = t[j];
    for (int o = 32; o > 0; o >>= 1) {
      x += __shfl_down(x, o, 64);
      y += __shfl_down(y, o, 64);
    }
    if (lane == 0) s_red[j][wv] = x;
    __syncthreads();
    off[j] = s_red[j][0] + s_red[j][1] + s_red[j][2] + s_red[j][3];
    __syncthreads();
    if (lane == 0) s_red[j][wv] = y;
    __syncthreads();
    tot[j] = s_red[j][0] + s_red[j][1] + s_red[j][2] + s_red[j][3];
    __syncthreads();
  }
  const int base = m.counters[kCntNew], sbase = m.counters[kCntSlideBase];
  const int i0 = blockIdx.x * kRootTile;
  for (int i = i0 + threadIdx.x; i < min(n, i0 + kRootTile); i += blockDim.x) {
    const uint32_t rk = rank[i];
    const int code = (int)(rk >> 29);
    if (!(code & 1)) continue;
    const uint32_t s = hslot[i];
    int r;
    if (code & 2) {  // a new root (voxel_map.cpp:77-83): centre, quater_length, empty records
      r = base + off[1] + (int)(rk & 0xffffu);
      if (r >= m.cap_nodes) {
        atomicOr(&m.counters[kCntErr], 4);
        continue;
      }
      const uint64_t key = m.hkey[s];
      double c[3];
      const int64_t k[3] = {unpack_axis(key, 42), unpack_axis(key, 21), unpack_axis(key, 0)};
      for (int j = 0; j < 3; j++) c[j] = (0.5 + k[j]) * mp.vs;
      init_node(m.hdr[r], c, (float)(mp.vs / 4.0), 0, -1);  // records zeroed by map_reset
      dbox_root(m.dbox + (size_t)r * 6);
      m.hval[s] = r;
    } else {
      r = m.hval[s];
      m.hdr[r].isexist = 1;
    }
    if (code & 4) {
      m.in_slide[r] = 1;
      m.slide[sbase + off[2] + (int)((rk >> 16) & 0x1fffu)] = r;
    }
    m.hfirst[s] = 0x7f7f7f7f;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    m.counters[kCntNodes] = min(base + tot[1], m.cap_nodes);
    m.counters[kCntRoots] = tot[1];
    m.counters[kCntTouched] = tot[0];
    m.counters[kCntSlide] = sbase + tot[2];
  }
}

// Root registration in ONE launch (k_ins_flags + k_ins_roots_alloc): each
// 1024-point tile publishes its three counts (first points, new roots, slide
// joiners) as one 64-bit granule {valid bit, 3 x 21-bit counts} with an
// agent-scope store, then sums the granules of the tiles before it (decoupled
// look-back: tiles are dispatched in order per XCD, so a tile only ever waits
// for tiles already dispatched) and allocates its own roots at base + prefix —
// the same ids and slide positions as the two-launch form. The granules are
// zeroed by k_ins_prep, the launch before. The last tile writes the totals.
__global__ void __launch_bounds__(256) k_ins_roots_lb(int n_arg, const int* __restrict__ nd, int ntile,
                                                      const uint32_t* __restrict__ hslot, MP mp, DevMap m,
                                                      unsigned long long* __restrict__ gran) {
  const int n = nd ? *nd : n_arg;
  __shared__ u64 s_w[4];
  __shared__ int s_off[3], s_tot[3];
  const int tid = threadIdx.x, lane = tid & 63, b = blockIdx.x;
  const int i0 = b * kRootTile + tid * 4;
  int code[4];
  u64 v = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    code[k] = ins_root_code(m, hslot, i0 + k, n);
    v += pack3(code[k]);
  }
  u64 tot;
  u64 r = block_excl_scan3(v, s_w, &tot);
  constexpr u64 kF = (1ull << 21) - 1;
  if (tid == 0) __hip_atomic_store(&gran[b], tot | (1ull << 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid < 64) {  // wave 0: the earlier tiles' counts (and, in the last tile, everyone's)
    const bool last = b == ntile - 1;
    const int upto = last ? ntile : b;
    int a0 = 0, a1 = 0, a2 = 0, t0 = 0, t1 = 0, t2 = 0;
    for (int k = lane; k < upto; k += 64) {
      u64 g;
      for (long it = 0;; it++) {
        g = __hip_atomic_load(&gran[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (g >> 63) break;
        __builtin_amdgcn_s_sleep(1);
        if (it > (1l << 24)) {  // never: a tile that never publishes (bounded, not a hang)
          atomicOr(&m.counters[kCntErr], 64);
          g = 1ull << 63;
          break;
        }
      }
      const int c0 = (int)(g & kF), c1 = (int)((g >> 21) & kF), c2 = (int)((g >> 42) & kF);
      if (k < b) {
        a0 += c0;
        a1 += c1;
        a2 += c2;
      }
      t0 += c0;
      t1 += c1;
      t2 += c2;
    }
    for (int o = 32; o > 0; o >>= 1) {
      a0 += __shfl_down(a0, o, 64);
      a1 += __shfl_down(a1, o, 64);
      a2 += __shfl_down(a2, o, 64);
      t0 += __shfl_down(t0, o, 64);
      t1 += __shfl_down(t1, o, 64);
      t2 += __shfl_down(t2, o, 64);
    }
    if (lane == 0) {
      s_off[0] = a0;
      s_off[1] = a1;
      s_off[2] = a2;
      s_tot[0] = t0;
      s_tot[1] = t1;
      s_tot[2] = t2;
    }
  }
  __syncthreads();
  const int base = m.counters[kCntNew], sbase = m.counters[kCntSlideBase];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int i = i0 + k;
    const int cd = code[k];
    const u64 rk = r;
    r += pack3(cd);
    if (i >= n || !(cd & 1)) continue;
    const uint32_t s = hslot[i];
    int rt;
    if (cd & 2) {  // a new root (voxel_map.cpp:77-83): centre, quater_length, empty records
      rt = base + s_off[1] + (int)((rk >> 21) & kF);
      if (rt >= m.cap_nodes) {
        atomicOr(&m.counters[kCntErr], 4);
        continue;
      }
      const uint64_t key = m.hkey[s];
      double c[3];
      const int64_t kk[3] = {unpack_axis(key, 42), unpack_axis(key, 21), unpack_axis(key, 0)};
      for (int j = 0; j < 3; j++) c[j] = (0.5 + kk[j]) * mp.vs;
      init_node(m.hdr[rt], c, (float)(mp.vs / 4.0), 0, -1);  // records zeroed by map_reset
      dbox_root(m.dbox + (size_t)rt * 6);
      m.hval[s] = rt;
    } else {
      rt = m.hval[s];
      m.hdr[rt].isexist = 1;
    }
    if (cd & 4) {
      m.in_slide[rt] = 1;
      m.slide[sbase + s_off[2] + (int)((rk >> 42) & kF)] = rt;
    }
    m.hfirst[s] = 0x7f7f7f7f;
  }
  if (b == ntile - 1 && tid == 0) {
    m.counters[kCntNodes] = min(base + s_tot[1], m.cap_nodes);
    m.counters[kCntRoots] = s_tot[1];
    m.counters[kCntTouched] = s_tot[0];
    m.counters[kCntSlide] = sbase + s_tot[2];
  }
}

// allocate new roots in first-occurrence order (deterministic ids); new roots
// join surf_map_slide (voxel_map.cpp:77-83)
__global__ void __launch_bounds__(256) k_ins_newalloc(int n, const uint32_t* __restrict__ hslot, const uint32_t* __restrict__ flag,
                               const uint32_t* __restrict__ rank, MP mp, DevMap m) {
  const int base = m.counters[kCntNodes];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (!flag[i]) continue;
    uint32_t s = hslot[i];
    int id = base + (int)rank[i];
    if (id >= m.cap_nodes) {
      atomicOr(&m.counters[kCntErr], 4);
      continue;
    }
    uint64_t key = m.hkey[s];
    double c[3];
    int64_t k[3] = {unpack_axis(key, 42), unpack_axis(key, 21), unpack_axis(key, 0)};
    for (int j = 0; j < 3; j++) c[j] = (0.5 + k[j]) * mp.vs;
    init_node(m.hdr[id], c, (float)(mp.vs / 4.0), 0, -1);
    dbox_root(m.dbox + (size_t)id * 6);
    m.hval[s] = id;
    m.hfirst[s] = 0x7f7f7f7f;
    m.in_slide[id] = 1;
    int pos = atomicAdd(&m.counters[kCntSlide], 1);
    m.slide[pos] = id;
  }
}

__global__ void __launch_bounds__(256) k_add_counter(int* counters, int idx, const uint32_t* __restrict__ flag,
                              const uint32_t* __restrict__ rank, int n) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && n > 0) counters[idx] += (int)(rank[n - 1] + flag[n - 1]);
}

// distinct roots touched by the scan (the thread_num quirk, voxel_map.cpp:94-97),
// isexist on existing roots (voxel_map.cpp:70), surf_map_slide registration
__global__ void __launch_bounds__(256) k_ins_touch(int n, const uint32_t* __restrict__ hslot, int epoch, DevMap m,
                           int* __restrict__ root_of) {
  const int first_new = m.counters[kCntNew];
  for (int base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
    const int i = base + threadIdx.x;
    int first = 0, add_slide = 0, root = -1;
    if (i < n) {
      uint32_t s = hslot[i];
      root = s != 0xffffffffu ? m.hval[s] : -1;
      root_of[i] = root;
      if (root >= 0 && atomicExch(&m.nscr[(size_t)root * 4 + 3], epoch) != epoch) {
        first = 1;
        if (root < first_new) {
          m.hdr[root].isexist = 1;
          if (!m.in_slide[root]) {
            m.in_slide[root] = 1;
            add_slide = 1;
          }
        }
      }
    }
    (void)wave_append(&m.counters[kCntTouched], first);
    int pos = wave_append(&m.counters[kCntSlide], add_slide);
    if (add_slide) m.slide[pos] = root;
  }
}

// descend to a leaf; a missing child becomes a creation request (parent, octant)
// the later insert kernels do nothing when the scan touched fewer than
// thread_num roots (voxel_map.cpp:96-97: no allocation at all) or when the
// child allocation overflowed k_ins_alloc (the host replays them)
__device__ __forceinline__ bool ins_skip(const DevMap& m, int thread_num) {
  return g_touched(m) < thread_num || m.counters[kCntMisc] != 0;
}

__global__ void k_copy_int(const int* __restrict__ src, int* __restrict__ dst) {
  if (threadIdx.x == 0) *dst = *src;
}

__global__ void __launch_bounds__(256) k_ins_descend(int n_arg, const int* __restrict__ nd, int thread_num, const double* __restrict__ pw, DevMap m,
                                                     const uint32_t* __restrict__ hslot, int* __restrict__ leaf,
                                                     int* __restrict__ reqlist) {
  const int n = nd ? *nd : n_arg;  // the downsampled count on the device (ds_enqueue_hashed)
  if (ins_skip(m, thread_num)) return;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t hs = hslot[i];
    int node = hs != 0xffffffffu ? m.hval[hs] : -1;  // the point's root (registered by k_ins_roots_alloc)
    leaf[i] = node;
    if (node < 0) continue;
    V3 w = v3(pw[3 * i], pw[3 * i + 1], pw[3 * i + 2]);
    for (int d = 0; d < 8; d++) {
      const NodeHdr& h = m.hdr[node];
      if (h.octo == 0) break;
      int o = octant(w, h.center);
      int c = h.child[o];
      if (c < 0) {
        // request (parent, octant); the first requester of a parent registers it
        if (atomicCAS(&m.cfirst[(size_t)node * 8 + o], 0x7f7f7f7f, -5) == 0x7f7f7f7f) {
          if (atomicExch(&m.nscr[(size_t)node * 4 + 1], -7) != -7) {
            int pos = atomicAdd(&m.counters[kCntCreate], 1);
            reqlist[pos] = node;
          }
        }
        node = -2 - (node * 8 + o);
        break;
      }
      node = c;
    }
    leaf[i] = node;
  }
}

// children for a sorted list of parents: ids = base + prefix(popcount(mask))
__global__ void __launch_bounds__(256) k_child_count(int np, const int* __restrict__ parents, DevMap m, uint32_t* __restrict__ cnt) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < np; q += gridDim.x * blockDim.x) {
    int p = parents[q];
    int c = 0;
    for (int o = 0; o < 8; o++) c += (m.cfirst[(size_t)p * 8 + o] == -5) ? 1 : 0;
    cnt[q] = (uint32_t)c;
  }
}

// One-wave workgroups for the thread-per-item kernels whose work covers fewer
// workgroups than the chip has CUs (k_ins_descend / resolve / scatter over a
// scan's points, k_rc_visit, k_collect_level, the margi passes): their
// scattered record loads (64 cache lines per instruction) then spread over 4x
// the CUs' address units instead of queueing four waves deep on a quarter of
// them (k_margi_leaf 37.7 -> 32.9 us, k_rc_visit 15.0 -> 13.2 us)
constexpr int kSpreadBlock = 64;

__global__ void __launch_bounds__(256) k_child_alloc(int np, const int* __restrict__ parents, const uint32_t* __restrict__ off, DevMap m,
                              int* __restrict__ next, int next_base);

// the final leaf of every point, and its bucket: a point count per leaf
// (m.leaf_cnt, zero between inserts) and, for the leaf's first point, a
// segment (seg_leaf[s] = leaf, m.leaf_seg[leaf] = s). Segment order is free:
// k_push_window treats every leaf on its own; only the order of a leaf's
// points matters, and k_push_window restores it.
__global__ void __launch_bounds__(256) k_ins_resolve(int n_arg, const int* __restrict__ nd, int thread_num, const double* __restrict__ pw, DevMap m,
                                                     int* __restrict__ leaf, int* __restrict__ seg_leaf) {
  const int n = nd ? *nd : n_arg;  // the downsampled count on the device (ds_enqueue_hashed)
  if (ins_skip(m, thread_num)) return;
  for (int base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
    const int i = base + threadIdx.x;
    int node = i < n ? leaf[i] : -1;
    if (node < -1) {
      const int code = -2 - node;
      node = m.hdr[code >> 3].child[code & 7];
      leaf[i] = node;
    }
    const bool first = node >= 0 && atomicAdd(&m.leaf_cnt[node], 1) == 0;
    const int s = wave_append(&m.counters[kCntSeg], first ? 1 : 0);
    if (first) {
      seg_leaf[s] = node;
      m.leaf_seg[node] = s;
    }
  }
}

// one workgroup: segment offsets = prefix over the segments' point counts;
// the counts return to zero (k_ins_scatter counts the fill again)
__global__ void __launch_bounds__(1024) k_seg_offsets(int thread_num, DevMap m, const int* __restrict__ seg_leaf,
                                                      int* __restrict__ seg_off) {
  __shared__ int s_w[17];
  if (ins_skip(m, thread_num)) return;
  const int ns = m.counters[kCntSeg];
  const int per = (ns + (int)blockDim.x - 1) / (int)blockDim.x;
  const int s0 = threadIdx.x * per, s1 = min(ns, s0 + per);
  constexpr int kPer = 32;
  int total;
  if (per <= kPer) {  // all loads of a lane issued before any is used (two round trips, not 2 per segment)
    int lf[kPer], c[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) lf[k] = s0 + k < s1 ? seg_leaf[s0 + k] : -1;
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      c[k] = lf[k] >= 0 ? m.leaf_cnt[lf[k]] : 0;
      cnt += c[k];
    }
    int pos = block_excl_scan(cnt, s_w, &total);
#pragma unroll
    for (int k = 0; k < kPer; k++)
      if (lf[k] >= 0) {
        seg_off[s0 + k] = pos;
        pos += c[k];
        m.leaf_cnt[lf[k]] = 0;
      }
  } else {
    int cnt = 0;
    for (int q = s0; q < s1; q++) cnt += m.leaf_cnt[seg_leaf[q]];
    int pos = block_excl_scan(cnt, s_w, &total);
    for (int q = s0; q < s1; q++) {
      const int l = seg_leaf[q];
      seg_off[q] = pos;
      pos += m.leaf_cnt[l];
      m.leaf_cnt[l] = 0;
    }
  }
  if (threadIdx.x == 0) seg_off[ns] = total;
}

// every point into its segment (arbitrary order inside it)
__global__ void __launch_bounds__(256) k_ins_scatter(int n_arg, const int* __restrict__ nd, int thread_num, DevMap m, const int* __restrict__ leaf,
                                                     const int* __restrict__ seg_off, int* __restrict__ order) {
  const int n = nd ? *nd : n_arg;  // the downsampled count on the device (ds_enqueue_hashed)
  if (ins_skip(m, thread_num)) return;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int l = leaf[i];
    if (l < 0) continue;
    order[seg_off[m.leaf_seg[l]] + atomicAdd(&m.leaf_cnt[l], 1)] = i;
  }
}

// pvec_update into the leaves (voxel_map.cpp:104-131 / octree.cpp:151-177):
// one wave per leaf segment (k_ins_resolve / k_seg_offsets / k_ins_scatter);
// lanes 0-8 own the frame cluster, 9-17 the accumulated cluster, 18-62
// cov_add (see role_inc)
constexpr int kPushWaves = 4;
constexpr int kPwBits = 1 << 16;  // point indices per bitmap window of k_push_window (8 KB, inside the wave's E)
constexpr int kPwWords = kPwBits / 32;
constexpr int kPwRankMax = 256;  // longest segment ordered by ranking (the bitmap's cost is its index range)
static_assert(kPwWords * 4 <= 64 * kErec * 8, "the ordering bitmap lives in the wave's record buffer");
// the recut's head (k_make_win_recut_begin's work) riding in the insert's
// last launch as one extra workgroup: the window view and the level counters
// need only the insert's counts, and the recut's first level starts one launch
// boundary earlier (the insert + recut graph, map_insert's rb)
struct RcBeginArg {
  WinArg wa;
  DState* st;
  const int* wpn;
  WinD* win;
  int* nper;
  int* slot_of;
  int* rc;
};
__device__ __forceinline__ void recut_begin_block(DevMap& m, int* __restrict__ rc, int thread_num);
__global__ void __launch_bounds__(64 * kPushWaves, 4) k_push_window(const int* __restrict__ seg_leaf,
                                                                 const int* __restrict__ seg_off,
                                                                 const int* __restrict__ order,
                                                                 int* __restrict__ order2, MP mp, int slot, DevMap m,
                                                                 const double* __restrict__ pw, int thread_num,
                                                                 RcBeginArg rb, int has_rb) {
  __shared__ double E[kPushWaves][64][kErec];
  if (has_rb && blockIdx.x == gridDim.x - 1) {
    make_win_block(rb.st, rb.wa, rb.wpn, rb.win, rb.nper, rb.slot_of);
    __syncthreads();
    recut_begin_block(m, rb.rc, thread_num);
    return;
  }
  if (ins_skip(m, thread_num)) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int role = lane < 63 ? lane : -1;
  RoleIdx ri = role < 9 ? role_clu(role < 0 ? 0 : role, kEq) : role < 18 ? role_clu(role - 9, kEp) : role_cov(role - 18);
  const int nseg = m.counters[kCntSeg];
  const int gsz = (int)gridDim.x - (has_rb ? 1 : 0);
  for (int sg = blockIdx.x * kPushWaves + wv; sg < nseg; sg += gsz * kPushWaves) {
    const int j0 = seg_off[sg], L = seg_off[sg + 1] - j0;
    const int leaf = seg_leaf[sg];
    // the leaf's points in index order (the reference's push order): up to 64
    // sorted across the lanes (bitonic by xor shuffles), longer segments ranked
    // into order2
    int mine = lane < L ? order[j0 + lane] : 0x7fffffff;
    if (L <= 64) {
#pragma unroll
      for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
          const int other = __shfl_xor(mine, j, 64);
          const bool up = (lane & k) == 0, low = (lane & j) == 0;
          mine = (low == up) ? min(mine, other) : max(mine, other);
        }
    } else if (L <= kPwRankMax) {  // a few hundred points: each ranked against the (L1-resident) others
      for (int e = lane; e < L; e += 64) {
        const int x = order[j0 + e];
        int r = 0;
        for (int t = 0; t < L; t++) r += order[j0 + t] < x ? 1 : 0;
        order2[j0 + r] = x;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
      // longer segments: an LDS bitmap over the segment's index range, in
      // windows of kPwBits indices (set bits compacted in order by a wave
      // scan): O(L + range / 32) per leaf instead of ranking every point
      // against every other (O(L^2 / 64) global loads per lane)
      uint32_t* bm = reinterpret_cast<uint32_t*>(&E[wv][0][0]);  // free until the records are filled
      int lo = 0x7fffffff, hi = -1;
      for (int e = lane; e < L; e += 64) {
        const int x = order[j0 + e];
        lo = min(lo, x);
        hi = max(hi, x);
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, __shfl_xor(lo, off, 64));
        hi = max(hi, __shfl_xor(hi, off, 64));
      }
      int outpos = 0;
      for (int w0 = lo; w0 <= hi; w0 += kPwBits) {
        const int nw = min(kPwWords, ((hi - w0) >> 5) + 1);  // the words this window's range covers
        for (int k = lane; k < nw; k += 64) bm[k] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        for (int e = lane; e < L; e += 64) {
          const int off = order[j0 + e] - w0;
          if (off >= 0 && off < kPwBits) atomicOr(&bm[off >> 5], 1u << (off & 31));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        // 64 consecutive words per round, one per lane: a lane emits at
        // most 32 indices per round however the points cluster
        for (int r = 0; r < nw; r += 64) {
          const int k = r + lane;
          uint32_t w = k < nw ? bm[k] : 0u;
          const int cnt = __popc(w);
          int ex = cnt;
#pragma unroll
          for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(ex, off, 64);
            if (lane >= off) ex += y;
          }
          int pos = outpos + ex - cnt;
          while (w) {
            const int b = __ffs(w) - 1;
            w &= w - 1;
            order2[j0 + pos++] = w0 + k * 32 + b;
          }
          outpos += __shfl(ex, 63, 64);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      }
    }
    const bool listed = m.hdr[leaf].layer < mp.max_layer;
    if (listed) {  // the leaf's run of this slot (index order), for the recut's subdivisions and the margi
      int* ord = m.wp_ord + (size_t)slot * m.ord_stride + j0;
      if (L <= 64) {
        if (lane < L) ord[lane] = mine;
      } else {
        for (int e = lane; e < L; e += 64) ord[e] = order2[j0 + e];
      }
      if (lane == 0) m.lseg[(size_t)leaf * mp.W + slot] = lseg_pack(j0, L, m.slot_epoch[slot]);
    }
    Clu* loc = &m.pcrs[(size_t)leaf * mp.W + slot];
    Clu* add = &m.pcr_add[leaf];
    double* acc_p = role < 0 ? nullptr
                    : role < 9 ? (role < 6 ? &loc->P[role] : &loc->v[role - 6])
                    : role < 18 ? (role < 15 ? &add->P[role - 9] : &add->v[role - 15])
                                : &m.cov_add[(size_t)leaf * kCovN + role - 18];
    double acc = acc_p ? *acc_p : 0.0;
    for (int base = 0; base < L; base += 64) {
      const int e = base + lane;
      const bool valid = e < L;
      if (valid) {
        const int i = L <= 64 ? mine : order2[j0 + e];
        const size_t b = (size_t)slot * m.cap_wp + i;
        fill_record(E[wv][lane], ld_v3(&m.wp_pnt[b * 3]), v3(pw[3 * i], pw[3 * i + 1], pw[3 * i + 2]),
                    ld_m3(&m.wp_var[b * 9]));
        if (listed) m.wp_leaf[b] = leaf;
      }
      const int nb = min(64, L - base);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 8
      for (int k = 0; k < nb; k++) acc += role_inc(E[wv][k], ri);  // unrolled: the LDS reads run ahead of the sum
      __builtin_amdgcn_wave_barrier();
    }
    if (acc_p) *acc_p = acc;
    if (lane == 0) {
      loc->N += L;
      add->N += L;
      m.hdr[leaf].has_sw = 1;
      m.hdr[leaf].isexist = 1;
      m.leaf_cnt[leaf] = 0;  // bucketing invariant: zero between inserts
    }
  }
}

// zero a freshly allocated node's records (the pool is zeroed lazily)
// children of parent p in octant order, ids id0, id0+1, ...; appended to next
__device__ __forceinline__ void alloc_parent(DevMap& m, int p, int id0, int* next, int next_pos) {
  NodeHdr& ph = m.hdr[p];
  int k = 0;
  for (int o = 0; o < 8; o++) {
    if (m.cfirst[(size_t)p * 8 + o] != -5) continue;
    const int id = id0 + k;
    k++;
    m.cfirst[(size_t)p * 8 + o] = 0x7f7f7f7f;
    if (id >= m.cap_nodes) {
      atomicOr(&m.counters[kCntErr], 4);
      continue;
    }
    int xyz[3] = {(o >> 2) & 1, (o >> 1) & 1, o & 1};
    double c[3];
    for (int j = 0; j < 3; j++) c[j] = ph.center[j] + (float)((2 * xyz[j] - 1) * ph.qlen);
    init_node(m.hdr[id], c, ph.qlen / 2, ph.layer + 1, p);
    dbox_child(m.dbox + (size_t)id * 6, m.dbox + (size_t)p * 6, ph.center, o);
    ph.child[o] = id;
    if (next) next[next_pos + k - 1] = id;
  }
  m.nscr[(size_t)p * 4 + 1] = -1;
}

// ascending bitonic sort of n (power of two) keys in LDS by the whole workgroup
template <typename T>
__device__ void lds_bitonic(T* a, int n) {
  for (int k = 2; k <= n; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int pj = i ^ j;
        if (pj > i) {
          const T x = a[i], y = a[pj];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            a[i] = y;
            a[pj] = x;
          }
        }
      }
      __syncthreads();
    }
}

// new roots: advance the node counter by the first-occurrence count
__global__ void k_ins_roots(DevMap m, const uint32_t* __restrict__ flag, const uint32_t* __restrict__ rank, int n) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const int c = n > 0 ? (int)(rank[n - 1] + flag[n - 1]) : 0;
    m.counters[kCntNodes] += c;
    m.counters[kCntRoots] = c;
  }
}

// children requested by k_ins_descend, in one workgroup: parents sorted
// ascending (deterministic ids), per-parent octant order, ids base + prefix,
// records zeroed. More than kInsAllocCap parents sets the abort flag and the
// host replays the allocation on the host-sized path.
constexpr int kInsAllocCap = 4096;
__global__ void __launch_bounds__(1024) k_ins_alloc(int thread_num, DevMap m, const int* __restrict__ reqlist,
                                                    int cap) {
  __shared__ int sp[kInsAllocCap];
  __shared__ int s_w[17];
  if (g_touched(m) < thread_num) return;
  const int np = m.counters[kCntCreate];
  if (np == 0) return;
  if (np > cap) {
    if (threadIdx.x == 0) m.counters[kCntMisc] = 1;
    return;
  }
  int npad = 2;
  while (npad < np) npad <<= 1;
  for (int i = threadIdx.x; i < npad; i += blockDim.x) sp[i] = i < np ? reqlist[i] : 0x7fffffff;
  __syncthreads();
  lds_bitonic(sp, npad);
  const int base = m.counters[kCntNodes];
  int carry = 0;
  for (int start = 0; start < np; start += blockDim.x) {
    const int q = start + threadIdx.x;
    const int p = q < np ? sp[q] : -1;
    int cc = 0;
    if (p >= 0)
      for (int o = 0; o < 8; o++) cc += (m.cfirst[(size_t)p * 8 + o] == -5) ? 1 : 0;
    int tot;
    const int off = block_excl_scan(cc, s_w, &tot);
    if (p >= 0) alloc_parent(m, p, base + carry + off, nullptr, 0);
    carry += tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) m.counters[kCntNodes] = base + carry;
}

static int read_counters(vg_ctx* ctx) {
  VG_HIP(hipMemcpyAsync(ctx->h_pinned, ctx->map.counters, kCntN * sizeof(int), hipMemcpyDeviceToHost,
                        ctx->stream));
  VG_HIP(stream_wait(ctx));
  if (ctx->h_pinned[kCntErr]) {
    int e = ctx->h_pinned[kCntErr];
    ctx->err = std::string("device map error flags=") + std::to_string(e) +
               ((e & 4) ? " (node pool full)" : "") + ((e & 8) ? " (point_fix arena full)" : "") +
               ((e & 1) ? " (voxel key out of packed range)" : "") + ((e & 2) ? " (root hash full)" : "") +
               ((e & 16) ? " (subdivision event buffer full)" : "");
    return (e & 1) ? VG_E_RANGE : VG_E_CAPACITY;
  }
  return VG_OK;
}

// LSD radix sort of 64-bit keys over bits [begin_bit, end_bit). The sort is
// stable, so keys (leaf << 27 | index) generated in index order need only
// their leaf bits sorted (3 passes instead of 7) to come out ordered by
// (leaf, index).
static int excl_scan(vg_ctx* ctx, const uint32_t* in, uint32_t* out, int n) {
  size_t tb = ctx->wk.tmp_bytes;
  if (n <= 0) return VG_OK;
  VG_HIP(hipcub::DeviceScan::ExclusiveSum(ctx->wk.tmp, tb, in, out, n, ctx->stream));
  return VG_OK;
}
static int bits_for(long v) {
  int b = 1;
  while ((1L << b) <= v) b++;
  return b;
}

// sort a list of n (non-negative) node ids, ascending (deterministic creation
// order), over the id bits only; returns the buffer holding the result (`a` or
// the scratch w.u1 — k0/k1 may hold live events)
static int sort_ids(vg_ctx* ctx, int* a, int n, int** result) {
  *result = a;
  if (n <= 1) return VG_OK;
  Work& w = ctx->wk;
  hipcub::DoubleBuffer<uint32_t> db(reinterpret_cast<uint32_t*>(a), w.u1);
  size_t tb = w.tmp_bytes;
  VG_HIP(hipcub::DeviceRadixSort::SortKeys(w.tmp, tb, db, n, 0, bits_for(ctx->map.cap_nodes), ctx->stream));
  *result = reinterpret_cast<int*>(db.Current());
  return VG_OK;
}
// in place
static int sort_ids_inplace(vg_ctx* ctx, int* a, int n) {
  int* r = a;
  VG_TRY(sort_ids(ctx, a, n, &r));
  if (r != a) VG_HIP(hipMemcpyAsync(a, r, (size_t)n * sizeof(int), hipMemcpyDeviceToDevice, ctx->stream));
  return VG_OK;
}

// allocate children for the parents in plist (sorted), ids deterministic
static int alloc_children(vg_ctx* ctx, int* plist, int np, int* next, int next_base, bool sorted, int* n_created) {
  Work& w = ctx->wk;
  hipStream_t s = ctx->stream;
  *n_created = 0;
  if (np <= 0) return VG_OK;
  if (!sorted) VG_TRY(sort_ids_inplace(ctx, plist, np));
  VG_TRY(read_counters(ctx));
  int first = ctx->h_pinned[kCntNodes];
  k_child_count<<<grid_for(np), kBlock, 0, s>>>(np, plist, ctx->map, w.ac_cnt);
  VG_TRY(excl_scan(ctx, w.ac_cnt, w.ac_off, np));
  k_child_alloc<<<grid_for(np), kBlock, 0, s>>>(np, plist, w.ac_off, ctx->map, next, next_base);
  k_add_counter<<<1, 64, 0, s>>>(ctx->map.counters, kCntNodes, w.ac_cnt, w.ac_off, np);
  VG_HIP(hipGetLastError());
  VG_TRY(read_counters(ctx));
  *n_created = ctx->h_pinned[kCntNodes] - first;
  return VG_OK;
}

// leaves -> sorted (leaf, order) keys -> pushes of one insert
static int insert_tail(vg_ctx* ctx, const MP& mp, int slot, int n, int thread_num, const int* nd = nullptr) {
  DevMap& m = ctx->map;
  Work& w = ctx->wk;
  hipStream_t s = ctx->stream;
  const int g = grid_for(n);
  const int gseg = (n + kPushWaves - 1) / kPushWaves < 2048 ? (n + kPushWaves - 1) / kPushWaves : 2048;
  int* seg_leaf = w.list1;
  int* seg_off = reinterpret_cast<int*>(w.v0);
  int* order = reinterpret_cast<int*>(w.k0);
  int* order2 = reinterpret_cast<int*>(w.k1);
  // leaves -> per-leaf buckets (no sort: the order between leaves is free)
  k_ins_resolve<<<g * (kBlock / kSpreadBlock), kSpreadBlock, 0, s>>>(n, nd, thread_num, w.pw, m, w.leaf, seg_leaf);
  k_seg_offsets<<<1, 1024, 0, s>>>(thread_num, m, seg_leaf, seg_off);
  k_ins_scatter<<<g * (kBlock / kSpreadBlock), kSpreadBlock, 0, s>>>(n, nd, thread_num, m, w.leaf, seg_off, order);
  // ~one wave per leaf segment (the count stays on the device); plus the
  // recut's head when the recut follows in the same graph (ctx->rc_begin_wa)
  RcBeginArg rb;
  memset(&rb, 0, sizeof(rb));
  const bool has_rb = ctx->rc_begin_wa != nullptr;
  if (has_rb) {
    rb.wa = *ctx->rc_begin_wa;
    rb.st = ctx->st;
    rb.wpn = m.wpn;
    rb.win = (WinD*)ctx->ba.xs;
    rb.nper = (int*)((char*)ctx->ba.xs + sizeof(WinD));
    rb.slot_of = rb.nper + 32;  // (map_recut's dslot)
    rb.rc = w.rc;
    ctx->rc_begin_wa = nullptr;
    ctx->rc_begun = true;
  }
  k_push_window<<<gseg + (has_rb ? 1 : 0), 64 * kPushWaves, 0, s>>>(seg_leaf, seg_off, order, order2, mp, slot, m, w.pw,
                                                                     thread_num, rb, has_rb ? 1 : 0);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

// cut_voxel_multi (voxel_map.cpp:47-135) + pvec_update (point_utils.cpp:54-65).
// Asynchronous: every count stays on the device. A child-allocation overflow
// of k_ins_alloc sets kCntMisc; the insert tail and the recut kernels then skip
// and map_recut reports it (kNeedInsertReplay) for map_insert_replay.
int map_insert(vg_ctx* ctx, const MP& mp, int slot, int n, int epoch, int thread_num, const PushArg* push,
               const InsPre* pre, const int* nd) {
  DevMap& m = ctx->map;
  Work& w = ctx->wk;
  hipStream_t s = ctx->stream;
  if (n <= 0) {
    if (push) VG_TRY(state_push(ctx, push->ord, push->new_imu, push->rec));
    return VG_OK;
  }
  // device count: n is an upper bound, the kernels stride over the real one
  const int g = nd ? grid_for(n, kBlock, 2048) : grid_for(n);
  if (pre)
    k_ins_prep<true><<<g, kBlock, 0, s>>>(n, nullptr, nullptr, nullptr, nullptr, nullptr, mp, ctx->st, slot, m, w.pw,
                                          w.u0,
                                          nullptr, pre->pnt, pre->pose, pre->var_identity, nullptr, w.gran, w.ngran,
                                          nullptr);
  else {
    // the push record goes through host-mapped memory, so a replayed graph
    // picks up each scan's record (the host writes it before the launch)
    // (slot in_sel: a scan graph's ring position, whose per-scan numbers ride along)
    HostIn* hin = ctx->h_in + ctx->in_sel;
    HostIn* din = ctx->d_in + ctx->in_sel;
    if (push) hin->push = *push;
    k_ins_prep<false><<<g, kBlock, 0, s>>>(n, nd, ctx->ds.ox, ctx->ds.oy, ctx->ds.oz, ctx->ds.oi, mp, ctx->st, slot, m,
                                           w.pw,
                                           w.u0, push ? &din->push : nullptr, nullptr, nullptr, 0,
                                           nd ? ctx->ds.hflags : nullptr, w.gran, w.ngran,
                                           ctx->in_ph ? din->ph : nullptr);
  }
  const int ntile = (n + kRootTile - 1) / kRootTile;
  (void)epoch;
  if (ctx->roots_lb && ntile <= w.ngran) {  // one launch (decoupled look-back)
    k_ins_roots_lb<<<ntile, kBlock, 0, s>>>(n, nd, ntile, w.u0, mp, m, w.gran);
  } else {
    k_ins_flags<<<ntile, kBlock, 0, s>>>(n, nd, w.u0, m, w.v1, (int*)w.ac_cnt);
    k_ins_roots_alloc<<<ntile, kBlock, 0, s>>>(n, nd, ntile, w.u0, w.v1, (const int*)w.ac_cnt, mp, m);
  }
  if (sharded(ctx)) {  // the thread_num quirk counts distinct roots over all shards
    VG_TRY(shard_allreduce(ctx, m.counters + kCntTouched, m.counters + kCntGTouched, 1, 1, 1));
  }
  k_ins_descend<<<g * (kBlock / kSpreadBlock), kSpreadBlock, 0, s>>>(n, nd, thread_num, w.pw, m, w.u0, w.leaf, w.list2);
  const int ins_cap = (ctx->dbg_ins_cap >= 0 && ctx->dbg_ins_cap < kInsAllocCap) ? ctx->dbg_ins_cap : kInsAllocCap;
  k_ins_alloc<<<1, 1024, 0, s>>>(thread_num, m, w.list2, ins_cap);
  return insert_tail(ctx, mp, slot, n, thread_num, nd);
}

// host-sized child allocation after a k_ins_alloc overflow, then the tail
int map_insert_replay(vg_ctx* ctx, const MP& mp, int slot, int n, int thread_num) {
  DevMap& m = ctx->map;
  hipStream_t s = ctx->stream;
  VG_TRY(read_counters(ctx));
  const int np = ctx->h_pinned[kCntCreate];
  VG_HIP(hipMemsetAsync(m.counters + kCntMisc, 0, sizeof(int), s));
  VG_HIP(hipMemsetAsync(m.counters + kCntSeg, 0, sizeof(int), s));
  int created = 0;
  VG_TRY(alloc_children(ctx, ctx->wk.list2, np, nullptr, 0, false, &created));
  return insert_tail(ctx, mp, slot, n, thread_num);
}

// ------------------------------------------------------------------ recut (A5/A6)
// Level-synchronous OctoTree::recut (octree.cpp:335-393) with every count kept
// on the device: per level, k_rc_visit (worklist -> children / subdividing
// leaves / factor candidates), k_rc_win (window points of subdividing leaves)
// and k_rc_apply (one workgroup: deterministic child allocation, event sort in
// LDS, pushes in the reference's order). The host enqueues max_layer+1 levels
// and synchronizes once. A level whose subdivision exceeds the LDS capacity of
// k_rc_apply sets rc[kRcAbort]; the host then replays the rest of the recut
// with the host-sized path (recut_slow_apply), which only happens while the
// map is first built.
constexpr int kApplyThreads = 1024;
constexpr int kApplySub = kApplyThreads;  // subdividing leaves per level (one lane each)

// visit one worklist entry; returns children / candidate / subdivide flags
__device__ __forceinline__ void recut_visit_node(int node, const MP& mp, DevMap& m, int* kids, int& nchild,
                                                 int& is_cand, int& is_sub) {
  nchild = 0;
  is_cand = 0;
  is_sub = 0;
  if (node < 0) return;
  NodeHdr& h = m.hdr[node];
  if (h.octo == 1) {
    for (int o = 0; o < 8; o++)
      if (h.child[o] >= 0) kids[nchild++] = h.child[o];
    return;
  }
  h.opt_state = -1;
  const Clu& a = m.pcr_add[node];
  if (a.N <= mp.minpt[h.layer]) {
    h.is_plane = 0;
  } else if (h.isexist && h.has_sw) {
    V3 ev;
    M3 U;
    eig3(clu_cov(a), ev, U);
    double* e = &m.eig[(size_t)node * 12];
    for (int j = 0; j < 3; j++) e[j] = ev[j];
    for (int j = 0; j < 9; j++) e[3 + j] = U[j];
    h.is_plane = (ev[0] < mp.min_eig && (ev[0] / ev[2]) < mp.thre[h.layer]) ? 1 : 0;
    if (h.is_plane) {
      is_cand = !(ev[0] / ev[1] > 0.12) ? 1 : 0;  // tras_opt filter, octree.cpp:502-505
    } else if (h.layer < mp.max_layer) {
      m.nscr[(size_t)node * 4 + 2] = 1;  // subdividing
      is_sub = 1;
    }
  }
}

__global__ void __launch_bounds__(256) k_rc_visit(int L, int thread_num, const int* __restrict__ work_in, MP mp,
                                                  DevMap m, int* __restrict__ next, int* __restrict__ sub,
                                                  int* __restrict__ cand, int* __restrict__ rc,
                                                  uint32_t* __restrict__ cand_bits) {
  if (rc[kRcAbort]) return;
  const int nw = (L == 0) ? m.counters[kCntSlide] : rc[kRcLvl + L - 1];
  if (L == 0 && g_slide(m) < thread_num) return;  // local_mapping.cpp:150-154 (global count)
  const int* work = (L == 0) ? m.slide : work_in;
  for (int base = blockIdx.x * blockDim.x; base < nw; base += gridDim.x * blockDim.x) {
    const int q = base + threadIdx.x;
    int kids[8], nchild, is_cand, is_sub;
    recut_visit_node(q < nw ? work[q] : -1, mp, m, kids, nchild, is_cand, is_sub);
    const int node = q < nw ? work[q] : -1;
    int o1, o2, o3;
    wave_append3(&rc[kRcLvl + L], nchild, &m.counters[kCntFactors], is_cand, &rc[kRcSub + L], is_sub, o1, o2, o3);
    for (int j = 0; j < nchild; j++) next[o1 + j] = kids[j];
    if (is_cand) {
      cand[o2] = node;
      if (cand_bits) atomicOr(&cand_bits[node >> 5], 1u << (node & 31));  // k_fac_sort's id order
    }
    if (is_sub) sub[o3] = node;
  }
}

// The points of every subdividing leaf (subdivide / fix_divide, octree.cpp:
// 257-300), one wave per leaf: its point_fix list, then its run of each
// window slot (DevMap::lseg) in frame order. Pass 1 finds each point's octant
// and counts per octant; pass 2 writes the events of each octant into their
// own range of the leaf's block of the event list, in walk order, so a child's
// events come out grouped and already in the reference's push order (point_fix
// by index, then frame by frame, index ascending) — no sort. Event: phase << 21
// | index (phase 0 point_fix, 1 + ord a window frame). rcinfo[18 q ..]: the
// block's start, then per octant its offset and count, then the mask of
// non-empty octants; nscr[leaf*4+0] = q.
constexpr int kRcWinWaves = 4;
constexpr int kRcWalkB = 4;  // rc_win_leaf: 64-point chunks per round of loads
constexpr int kRcInfo = 18;  // event base, 8 octant offsets, 8 octant counts, octant mask
// one wave per subdividing leaf: the leaf's points are flattened across the
// phases so each 64-point chunk costs one round of loads whatever the runs'
// lengths; pass 1 counts the octants, pass 2 writes each octant's events
// (ph << 21 | idx) at its running position, walk order kept. The leaf's
// children-to-be are counted into rc[kRcNch + L] (the fused level kernel
// sizes its pushes from it).
__device__ __forceinline__ void rc_win_leaf(int L, int leaf, int q, const WinD* __restrict__ win, DevMap& m,
                                            uint64_t* __restrict__ ev, int* __restrict__ rcinfo, int cap,
                                            int info_cap, int* __restrict__ rc) {
  const int lane = threadIdx.x & 63;
#ifdef VG_PROBE
  const unsigned long long wl_t0 = wall_clock64();  // scripts/probe_recut.py: 16-20 split time / points
#endif
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int wc = win->win_count;
  const int mp_l = win->mp[lane >= 1 && lane <= 32 ? lane - 1 : 0];  // in the same round of loads as wc
  const int my_slot = (lane >= 1 && lane <= wc) ? mp_l : 0;
  const NodeHdr& h = m.hdr[leaf];
  int len = 0, st = 0;
  if (lane == 0) len = h.fix_cnt;
  else if (lane <= wc && !lseg_get(m, leaf, my_slot, st, len)) len = 0;
  int ex = len;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(ex, off, 64);
    if (lane >= off) ex += y;
  }
  const int total = __shfl(ex, 63, 64);
  ex -= len;
  int base = 0;
  if (lane == 0) base = atomicAdd(&rc[kRcWin + L], total);
  base = __shfl(base, 0, 64);
  if ((size_t)q * kRcInfo + kRcInfo > (size_t)info_cap || base + total > cap) {
    if (lane == 0) {
      atomicOr(&m.counters[kCntErr], 16);
      if ((size_t)q * kRcInfo + kRcInfo <= (size_t)info_cap) rcinfo[(size_t)q * kRcInfo + 17] = 0;  // no children
    }
    return;
  }
  // kRcWalkB chunks of 64 walk points per round of loads (the index loads of
  // all of them, then all their point loads): a split costs two memory round
  // trips per batch instead of two per chunk; a leaf of at most one batch
  // keeps it in registers for pass 2
  constexpr int kB = kRcWalkB;
  int bph[kB], bix[kB], boc[kB];
  auto walk_batch = [&](int c0) __attribute__((always_inline)) {
    int loc[kB], pst[kB], psl[kB];
#pragma unroll
    for (int b = 0; b < kB; b++) {
      const int e = min((c0 + b) * 64 + lane, total - 1);
      int ph = 0;
#pragma unroll
      for (int step = 32; step >= 1; step >>= 1) {
        const int cand = ph + step;
        const int v = __shfl(ex, cand <= wc ? cand : wc, 64);
        if (cand <= wc && v <= e) ph = cand;
      }
      bph[b] = ph;
      loc[b] = e - __shfl(ex, ph, 64);
      pst[b] = __shfl(st, ph, 64);
      psl[b] = __shfl(my_slot, ph, 64);
      bix[b] = ph == 0 ? loc[b] : m.wp_ord[(size_t)psl[b] * m.ord_stride + pst[b] + loc[b]];
    }
#pragma unroll
    for (int b = 0; b < kB; b++) {
      const int ph = bph[b];
      const V3 pw = ph == 0 ? ld_v3(&m.fix_pnt[((size_t)h.fix_off + loc[b]) * 3])
                            : rigid(ld_m3(win->R[ph - 1]), ld_v3(&m.wp_pnt[((size_t)psl[b] * m.cap_wp + bix[b]) * 3]),
                                    ld_v3(win->p[ph - 1]));
      boc[b] = octant(pw, h.center);
    }
  };
  int cnt8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int c0 = 0; c0 * 64 < total; c0 += kB) {
    walk_batch(c0);
#pragma unroll
    for (int b = 0; b < kB; b++) {
      const int e = (c0 + b) * 64 + lane;
      int o = boc[b];
      if (e < total) m.cfirst[(size_t)leaf * 8 + o] = -5;
      else o = -1;
#pragma unroll
      for (int k = 0; k < 8; k++) cnt8[k] += __popcll(__ballot(o == k));
    }
  }
  int off8[8], run = 0, mask = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    off8[k] = run;
    run += cnt8[k];
    mask |= (cnt8[k] > 0) << k;
  }
  if (lane == 0) {
    int* inf = rcinfo + (size_t)q * kRcInfo;
    inf[0] = base;
    for (int k = 0; k < 8; k++) {
      inf[1 + k] = off8[k];
      inf[9 + k] = cnt8[k];
    }
    inf[17] = mask;
    m.nscr[(size_t)leaf * 4 + 0] = q;
    atomicAdd(&rc[kRcNch + L], __popc(mask));
  }
  const bool kept = total <= 64 * kB;  // pass 1's only batch is still in registers
  for (int c0 = 0; c0 * 64 < total; c0 += kB) {
    if (!kept) walk_batch(c0);
#pragma unroll
    for (int b = 0; b < kB; b++) {
      const int e = (c0 + b) * 64 + lane;
      const int o = e < total ? boc[b] : -1;
      int pos = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint64_t bk = __ballot(o == k);
        if (o == k) pos = base + off8[k] + __popcll(bk & below);
        off8[k] += __popcll(bk);
      }
      if (o >= 0) ev[pos] = ((uint64_t)bph[b] << 21) | (uint64_t)bix[b];
    }
  }
#ifdef VG_PROBE
  if (lane == 0) {
    const unsigned long long d = wall_clock64() - wl_t0;
    atomicMax(&g_probe[16], d);
    atomicAdd(&g_probe[17], d);
    atomicAdd(&g_probe[18], 1ull);
    atomicMax(&g_probe[19], (unsigned long long)total);
    atomicAdd(&g_probe[20], (unsigned long long)total);
  }
#endif
}
__global__ void __launch_bounds__(64 * kRcWinWaves) k_rc_win(int L, const int* __restrict__ sub,
                                                             const WinD* __restrict__ win, DevMap m,
                                                             uint64_t* __restrict__ ev, int* __restrict__ rcinfo,
                                                             int cap, int info_cap, int* __restrict__ rc) {
  if (rc[kRcAbort]) return;
  const int nsub = rc[kRcSub + L];
  if (win->win_count > 63) {
    if (threadIdx.x == 0 && blockIdx.x == 0) atomicOr(&m.counters[kCntErr], 16);
    return;
  }
  for (int q = blockIdx.x * kRcWinWaves + (threadIdx.x >> 6); q < nsub; q += gridDim.x * kRcWinWaves)
    rc_win_leaf(L, sub[q], q, win, m, ev, rcinfo, cap, info_cap, rc);
}

__global__ void __launch_bounds__(256) k_child_alloc(int np, const int* __restrict__ parents, const uint32_t* __restrict__ off, DevMap m,
                              int* __restrict__ next, int next_base) {
  const int base = m.counters[kCntNodes];
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < np; q += gridDim.x * blockDim.x)
    alloc_parent(m, parents[q], base + (int)off[q], next, next_base + (int)off[q]);
}

// finish a subdivided parent: release its SlideWindow, free point_fix,
// octo_state = 1 (octree.cpp:375-387)
__device__ __forceinline__ void sub_finish(DevMap& m, int p) {
  NodeHdr& h = m.hdr[p];
  h.has_sw = 0;
  for (int j = 0; j < m.W; j++) clu_zero(m.pcrs[(size_t)p * m.W + j]);
  h.fix_cnt = 0;
  h.fix_cap = 0;
  h.octo = 1;
  m.nscr[(size_t)p * 4 + 2] = -1;
}

// one workgroup: the subdividing leaves in ascending id order (deterministic
// child ids), their marked octants' children allocated as one block (base +
// prefix), each child's event range from k_rc_win's per-octant blocks
// (cseg), the parents finished. More subdividing leaves than the workgroup's
// lanes (or than the test knob sub_cap) hand the level to the host-sized path.
__device__ __forceinline__ void rc_child_segs(const DevMap& m, int p, int c0, const int* __restrict__ rcinfo,
                                              int* __restrict__ cseg) {
  const int* inf = rcinfo + (size_t)m.nscr[(size_t)p * 4 + 0] * kRcInfo;
  int k = 0;
  for (int o = 0; o < 8; o++) {
    if (m.hdr[p].child[o] < 0 || inf[9 + o] == 0) continue;
    cseg[2 * (c0 + k)] = inf[0] + inf[1 + o];
    cseg[2 * (c0 + k) + 1] = inf[0] + inf[1 + o] + inf[9 + o];
    k++;
  }
}
__global__ void __launch_bounds__(kApplyThreads) k_rc_apply(int L, int sub_cap, DevMap m, int* __restrict__ next,
                                                            const int* __restrict__ sub,
                                                            const int* __restrict__ rcinfo, int* __restrict__ cseg,
                                                            int* __restrict__ rc) {
  __shared__ int s_sub[kApplySub];
  __shared__ int s_wsum[32];
  const int tid = threadIdx.x;
  if (rc[kRcAbort]) return;
  const int nsub = rc[kRcSub + L];
  if (nsub == 0) return;
  VG_PROBE_BEGIN();
  if (nsub > sub_cap) {
    if (tid == 0) rc[kRcAbort] = L + 1;
    return;
  }
  int myp = tid < nsub ? sub[tid] : 0x7fffffff;
  {  // rank among the level's leaves, read from LDS (ids are distinct)
    __shared__ __attribute__((aligned(16))) int s_in[kApplySub];
    s_in[tid] = myp;
    __syncthreads();
    int rank = 0;
    if (tid < nsub) {
      const int4* v4 = reinterpret_cast<const int4*>(s_in);
      for (int q = 0; q < (nsub + 3) / 4; q++) {
        const int4 v = v4[q];
        rank += (v.x < myp) + (v.y < myp) + (v.z < myp) + (v.w < myp);
      }
    }
    __syncthreads();
    if (tid < nsub) s_sub[rank] = myp;
  }
  __syncthreads();
  const int p_t = tid < nsub ? s_sub[tid] : -1;
  int cc = 0;
  if (p_t >= 0)
    for (int o = 0; o < 8; o++) cc += (m.cfirst[(size_t)p_t * 8 + o] == -5) ? 1 : 0;
  int ntot;
  const int coff = block_excl_scan(cc, s_wsum, &ntot);
  const int base = m.counters[kCntNodes];
  const int nnext = rc[kRcLvl + L];
  __syncthreads();
  if (p_t >= 0) {
    alloc_parent(m, p_t, base + coff, next, nnext + coff);
    rc_child_segs(m, p_t, coff, rcinfo, cseg);
  }
  __syncthreads();
  if (tid == 0) {
    m.counters[kCntNodes] = base + ntot;
    rc[kRcLvl + L] = nnext + ntot;
    rc[kRcCh + L] = ntot;
    rc[kRcChBase + L] = base;
  }
  if (p_t >= 0) sub_finish(m, p_t);
  VG_PROBE_MARK(17);
#ifdef VG_PROBE
  if (tid == 0) atomicAdd(&g_probe[62], 1ull);
#endif
}

constexpr int kRcPushWaves = 4;
constexpr int kPushScan = 4;    // event batches a push scans in one round (rc_push_child)
constexpr int kPreN = 32 * 9;   // s_pre: the frame clusters' P/v, then their point counts
constexpr int kPreV = 5;        // s_pre values per lane (32 slots * 10 / 64)
// the pushes of one child (push_fix then push per frame, octree.cpp:151-188)
// by one wave: its events keys[j0, j1) (point_fix first, then frame by
// frame), its parent and layer given (the caller may have initialised the
// header in this same wave); E / s_slot / s_pre: the wave's LDS slices. Role
// layout: 0-8 accumulated cluster, 9-17 fixed cluster (point_fix events),
// 18-62 cov_add, 63-71 the frame cluster of the current window slot (lanes
// 0-7 carry a second role)
__device__ __forceinline__ void rc_push_child(int child, int parent, int layer, int j0, int j1,
                                              const uint64_t* __restrict__ keys, const MP& mp,
                                              const WinD* __restrict__ win, DevMap& m, double (*E)[kErec],
                                              int* s_slot, double* s_pre, const RoleIdx& ri0, const RoleIdx& ri1) {
  const int lane = threadIdx.x & 63;
  const int r0 = lane, r1 = lane + 64;
  const bool has1 = r1 < 72;
  NodeHdr& h = m.hdr[child];
  const NodeHdr& ph = m.hdr[parent];
  const bool listed = layer < mp.max_layer;
#ifdef VG_PROBE
  const bool pr = blockIdx.x == 0 && threadIdx.x == 0;  // workgroup 0's wave 0: 40 pushes, 41 events,
  unsigned long long pt0 = wall_clock64();              // 42 prologue, 43 batch loads, 44 serial sums
  if (pr) {
    atomicAdd(&g_probe[40], 1ull);
    atomicAdd(&g_probe[41], (unsigned long long)(j1 - j0));
  }
#define PUSH_MARK(k)                                    \
  do {                                                  \
    if (pr) {                                           \
      const unsigned long long n_ = wall_clock64();     \
      atomicAdd(&g_probe[(k)], n_ - pt0);               \
      pt0 = n_;                                         \
    }                                                   \
  } while (0)
#else
#define PUSH_MARK(k) (void)0
#endif
  // the child's events are phase << 21 | index, ascending: point_fix
  // (phase 0) first, then one contiguous run per window slot (phase 1 + ord).
  // Up to kPushScan batches are read in one round of loads and the runs are
  // counted with ballots; longer children binary-search the keys.
  const int nev = j1 - j0, wc = listed ? win->win_count : 0;
  // the prologue's other loads go out with the keys' (one round): each
  // lane's window slot and its epoch, the frame clusters (s_pre, stored
  // below) and the accumulators' starting values
  const int mp_l = win->mp[lane < 32 ? lane : 0];  // in the same round of loads as win_count
  const int my_slot = lane < win->win_count ? mp_l : 0;  // listed or not (the batches read it)
  const int my_epoch = lane < wc ? m.slot_epoch[my_slot] : 0;
  double pv[kPreV];
#pragma unroll
  for (int i = 0; i < kPreV; i++) {
    const int t = lane + 64 * i;
    pv[i] = 0.0;
    if (t < mp.W * 10) {
      const int sl = t < mp.W * 9 ? t / 9 : t - mp.W * 9, q = t < mp.W * 9 ? t % 9 : 9;
      const Clu& lc = m.pcrs[(size_t)child * mp.W + sl];
      pv[i] = q < 6 ? lc.P[q] : (q < 9 ? lc.v[q - 6] : (double)lc.N);
    }
  }
  auto acc_ptr = [&](int r, int slot) -> double* {
    if (r < 9) return r < 6 ? &m.pcr_add[child].P[r] : &m.pcr_add[child].v[r - 6];
    if (r < 18) return r < 15 ? &m.pcr_fix[child].P[r - 9] : &m.pcr_fix[child].v[r - 15];
    if (r < 63) return &m.cov_add[(size_t)child * kCovN + r - 18];
    Clu& lc = m.pcrs[(size_t)child * mp.W + slot];
    return r < 69 ? &lc.P[r - 63] : &lc.v[r - 69];
  };
  double a0 = r0 < 63 ? *acc_ptr(r0, 0) : 0.0, a1 = 0.0;
  const int n_add0 = lane == 0 ? m.pcr_add[child].N : 0, n_fix0 = lane == 0 ? m.pcr_fix[child].N : 0;
  int nfix = 0, run_lo = 0, run_n = 0;
  const bool short_ev = nev <= 64 * kPushScan;  // the keys stay in registers (kv) for the batches below
  uint64_t kv[kPushScan];
  if (short_ev) {
    int phv[kPushScan];
#pragma unroll
    for (int b = 0; b < kPushScan; b++) {
      const int e = 64 * b + lane;
      kv[b] = e < nev ? keys[j0 + e] : 0ull;
      phv[b] = e < nev ? (int)((kv[b] >> 21) & 63) : 64;
    }
#pragma unroll
    for (int b = 0; b < kPushScan; b++) nfix += __popcll(__ballot(phv[b] == 0));
    for (int q = 1, acc = nfix; q <= wc && acc < nev; q++) {
      int c = 0;
#pragma unroll
      for (int b = 0; b < kPushScan; b++) c += __popcll(__ballot(phv[b] == q));
      if (lane == q - 1) {
        run_lo = j0 + acc;
        run_n = c;
      }
      acc += c;
    }
  } else {
    for (int b0 = j0; b0 < j1; b0 += 64) {
      const int e = b0 + lane;
      const bool f = e < j1 && ((keys[e] >> 21) & 63) == 0;
      const int k = __popcll(__ballot(f));
      nfix += k;
      if (k < 64) break;
    }
    if (lane < wc) {
      auto lower = [&](uint64_t key) {
        int lo = j0, hi = j1;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (keys[mid] < key) lo = mid + 1;
          else hi = mid;
        }
        return lo;
      };
      run_lo = lower((uint64_t)(lane + 1) << 21);
      run_n = lower((uint64_t)(lane + 2) << 21) - run_lo;
    }
  }
  // the point_fix block and the slots' runs are allocated in one round (an
  // overflow of either fails the scan with VG_E_CAPACITY, so a run taken
  // beside a point_fix overflow is never used); the returning atomics are
  // consumed after the first batch's loads (settle), so their round trip
  // overlaps those loads
  int off = 0, run_st = 0;
  if (lane == 0 && nfix > 0 && listed) off = atomicAdd(&m.counters[kCntFix], nfix);
  if (lane < wc && run_n > 0) run_st = atomicAdd(&m.arena[my_slot], run_n);
  int fix_off = 0;
  bool settled = false;
  auto settle = [&]() __attribute__((always_inline)) {  // false: point_fix overflow (wave-uniform)
    settled = true;
    if (nfix > 0 && listed) {
      if (lane == 0) {
        if (off + nfix > m.cap_fix) {
          atomicOr(&m.counters[kCntErr], 8);
          off = -1;
        } else {
          h.fix_off = off;
          h.fix_cap = nfix;
          h.fix_cnt = nfix;
        }
      }
      fix_off = __shfl(off, 0, 64);
      if (fix_off < 0) return false;
    }
    // lane p < win_count holds phase p + 1's run in the slot's arena
    if (lane < wc && run_n > 0) {
      if (run_st + run_n > m.ord_stride) {
        atomicOr(&m.counters[kCntErr], 16);
        run_st = 0;
      } else {
        m.lseg[(size_t)child * mp.W + my_slot] = lseg_pack(run_st, run_n, my_epoch);
      }
    }
    // every slot's frame cluster, loaded above in one round (a slot's run is
    // contiguous, so each is read once, before this wave writes it): a
    // cluster switch then costs an LDS read, not a dependent HBM load; their
    // point counts sit at s_pre[kPreN + slot], so the count update at a
    // switch is a plain store
#pragma unroll
    for (int i = 0; i < kPreV; i++) {
      const int t = lane + 64 * i;
      if (t < mp.W * 10) s_pre[t < mp.W * 9 ? t : kPreN + t - mp.W * 9] = pv[i];
    }
    return true;
  };
  int cur_slot = -1, loc_n = 0, nwin = 0;
  PUSH_MARK(42);
  for (int b0 = j0; b0 < j1; b0 += 64) {
    const int e = b0 + lane, bi = (b0 - j0) >> 6;
    uint64_t k = 0ull;
    if (!short_ev) {
      k = e < j1 ? keys[e] : 0ull;
    } else {
#pragma unroll
      for (int b = 0; b < kPushScan; b++)  // (a register select: kv stays in VGPRs)
        if (bi == b) k = kv[b];
    }
    const int phase = (int)((k >> 21) & 63), idx = (int)(k & ((1u << 21) - 1));
    const int slot_e = __shfl(my_slot, phase > 0 ? phase - 1 : 0, 64);  // win->mp[phase - 1]
    V3 pt;
    M3 var;
    if (e < j1) {
      if (phase == 0) {
        const size_t f = (size_t)ph.fix_off + idx;
        pt = ld_v3(&m.fix_pnt[f * 3]);
        var = ld_m3(&m.fix_var[f * 9]);
        fill_record(E[lane], pt, pt, var);
        s_slot[lane] = -1;
      } else {
        const int ord = phase - 1, slot = slot_e;
        const size_t bb = (size_t)slot * m.cap_wp + idx;
        const V3 pnt = ld_v3(&m.wp_pnt[bb * 3]);
        fill_record(E[lane], pnt, rigid(ld_m3(win->R[ord]), pnt, ld_v3(win->p[ord])),
                    ld_m3(&m.wp_var[bb * 9]));
        s_slot[lane] = slot;
        m.wp_leaf[bb] = listed ? child : -1;
      }
    }
    if (!settled && !settle()) return;
    if (e < j1 && phase == 0 && listed) {  // the point_fix copy into the child's block
      const size_t d = (size_t)fix_off + (e - j0);
      for (int t = 0; t < 3; t++) m.fix_pnt[d * 3 + t] = pt[t];
      for (int t = 0; t < 9; t++) m.fix_var[d * 9 + t] = var[t];
    }
    if (listed) {  // the point into the child's run (ds_bpermute of the run's lane; uniform call)
      const int ph = e < j1 ? phase : 0;
      const int src = ph > 0 ? ph - 1 : 0;
      const int lo_p = __shfl(run_lo, src, 64), st_p = __shfl(run_st, src, 64);
      if (ph > 0) m.wp_ord[(size_t)slot_e * m.ord_stride + st_p + (e - lo_p)] = idx;
    }
    const int nb = (j1 - b0) < 64 ? (j1 - b0) : 64;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    PUSH_MARK(43);
#pragma unroll 4
    for (int k = 0; k < nb; k++) {
      const int slot = s_slot[k];
      const bool isfix = slot < 0;
      if (!isfix && slot != cur_slot) {  // frame cluster switch (uniform)
        if (cur_slot >= 0) {
          if (r0 >= 63) *acc_ptr(r0, cur_slot) = a0;
          if (has1) *acc_ptr(r1, cur_slot) = a1;
          if (lane == 63) m.pcrs[(size_t)child * mp.W + cur_slot].N = (int)s_pre[kPreN + cur_slot] + loc_n;
        }
        cur_slot = slot;
        if (r0 >= 63) a0 = s_pre[cur_slot * 9 + r0 - 63];
        if (has1) a1 = s_pre[cur_slot * 9 + r1 - 63];
        loc_n = 0;
      }
      const double* Ek = E[k];
      const bool use0 = r0 < 9 || (r0 >= 18 && r0 < 63) || (r0 < 18 ? isfix : !isfix);
      const double i0 = role_inc(Ek, ri0);
      if (use0) a0 += i0;
      if (has1 && !isfix) a1 += role_inc(Ek, ri1);
      if (!isfix) {
        loc_n++;
        nwin++;
      }
    }
    __builtin_amdgcn_wave_barrier();
    PUSH_MARK(44);
  }
#undef PUSH_MARK
  if (!settled && !settle()) return;  // no events
  if (r0 < 63) *acc_ptr(r0, 0) = a0;
  if (cur_slot >= 0) {
    if (r0 >= 63) *acc_ptr(r0, cur_slot) = a0;
    if (has1) *acc_ptr(r1, cur_slot) = a1;
    if (lane == 63) m.pcrs[(size_t)child * mp.W + cur_slot].N = (int)s_pre[kPreN + cur_slot] + loc_n;
  }
  if (lane == 0) {
    m.pcr_add[child].N = n_add0 + nev;
    m.pcr_fix[child].N = n_fix0 + nfix;
    if (nwin > 0) {
      h.has_sw = 1;
      h.isexist = 1;
    }
  }
}
__device__ __forceinline__ RoleIdx rc_push_role(int r) {
  if (r < 9) return role_clu(r, kEp);
  if (r < 18) return role_clu(r - 9, kEp);
  if (r < 63) return role_cov(r - 18);
  return role_clu(r - 63, kEq);
}

// pushes of one level's children, one wave per child (rc_push_child)
__global__ void __launch_bounds__(64 * kRcPushWaves) k_rc_push(int L, const uint64_t* __restrict__ keys,
                                                               const int* __restrict__ cseg, MP mp,
                                                               const WinD* __restrict__ win, DevMap m,
                                                               const int* __restrict__ rc) {
  __shared__ double E[kRcPushWaves][64][kErec];
  __shared__ int s_slot[kRcPushWaves][64];  // window slot of the event, -1 for point_fix
  __shared__ double s_pre[kRcPushWaves][32 * 10];  // the child's frame clusters, read ahead
  if (rc[kRcAbort]) return;
  const int nch = rc[kRcCh + L], cbase = rc[kRcChBase + L];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const RoleIdx ri0 = rc_push_role(lane), ri1 = rc_push_role(lane + 64 < 72 ? lane + 64 : 0);
  for (int c = blockIdx.x * kRcPushWaves + wv; c < nch; c += gridDim.x * kRcPushWaves) {
    const int child = cbase + c;
    const NodeHdr& h = m.hdr[child];
    rc_push_child(child, h.parent, h.layer, cseg[2 * c], cseg[2 * c + 1], keys, mp, win, m, E[wv], s_slot[wv],
                  s_pre[wv], ri0, ri1);
  }
}

// ---- the fused recut levels -------------------------------------------
// The level loop above costs four dependent launches per level (visit, win,
// apply, push). The fused form runs one launch per level boundary:
//   k_rc_level0   visit(0) + win(0): the slide roots, 64 per wave; each wave
//                 then splits the subdividing leaves its lanes found;
//   k_rc_level(L) apply(L) + push(L) + visit(L+1) + win(L+1): the level's
//                 subdividing leaves are sorted and their children counted in
//                 LDS by every workgroup that pushes (redundantly: the same
//                 ids k_rc_apply hands out, base + prefix in ascending parent
//                 id order, so node ids and every order derived from them are
//                 unchanged); one wave per child initialises it, pushes its
//                 events, visits it and, when it subdivides, splits its
//                 points for level L+1; the grid's last waves visit (and
//                 split) the level's other nodes, the children of internal
//                 nodes listed by visit(L).
// Level L's sub list / rcinfo / events and level L+1's live in alternate
// buffers (sub_of / info_of / ev_of), so one launch reads the first and
// writes the second. The node counter's value before the level is carried in
// rc (kRcNode0, then kRcChBase + kRcCh of the previous level), so no
// workgroup reads a counter another one advances. Abort and overflow
// semantics are the level loop's (rc[kRcAbort] = L + 1; the host-sized path
// replays from there).

// one wave: visit the list entries [64 j, 64 j + 64) of level L; appends the
// internal nodes' children to next, the candidates, the subdividing leaves
// to sub; then (do_win) splits each subdividing leaf (rc_win_leaf)
__device__ __forceinline__ void rc_visit_chunk(int L, const int* __restrict__ work, int nw, int j, const MP& mp,
                                               DevMap& m, int* __restrict__ next, int* __restrict__ sub,
                                               int* __restrict__ cand, int* __restrict__ rc,
                                               uint32_t* __restrict__ cand_bits, bool do_win,
                                               const WinD* __restrict__ win, uint64_t* __restrict__ ev,
                                               int* __restrict__ rcinfo, int cap) {
  const int q = j * 64 + (threadIdx.x & 63);
  const int node = q < nw ? work[q] : -1;
  int kids[8], nchild, is_cand, is_sub;
  recut_visit_node(node, mp, m, kids, nchild, is_cand, is_sub);
  int o1, o2, o3;
  wave_append3(&rc[kRcLvl + L], nchild, &m.counters[kCntFactors], is_cand, &rc[kRcSub + L], is_sub, o1, o2, o3);
  for (int k = 0; k < nchild; k++) next[o1 + k] = kids[k];
  if (is_cand) {
    cand[o2] = node;
    if (cand_bits) atomicOr(&cand_bits[node >> 5], 1u << (node & 31));  // k_fac_sort's id order
  }
  if (is_sub) sub[o3] = node;
  if (!do_win) return;
  uint64_t bs = __ballot(is_sub);
  while (bs) {
    const int l = __ffsll((unsigned long long)bs) - 1;
    bs &= bs - 1;
    rc_win_leaf(L, __shfl(node, l, 64), __shfl(o3, l, 64), win, m, ev, rcinfo, cap, cap, rc);
  }
}

constexpr int kRcFusedWaves = 4;
// in-kernel clock of the recut's level kernels (KClock rc_*, vg_profile bit 2)
__device__ __forceinline__ void rc_clock_start(KClock* clk) {
  if (clk && clk->on && blockIdx.x == 0 && threadIdx.x == 0) {
    const int slot = clk->scan & (kClkRcScans - 1);
    clk->rc_t0[slot] = (unsigned long long)wall_clock64();
    clk->rc_exec[slot] = 1;
  }
}
__device__ __forceinline__ void rc_clock_end(KClock* clk) {
  if (clk && clk->on && blockIdx.x < kClkRcBlocks) {
    __syncthreads();
    if (threadIdx.x == 0) clk->rc_tend[clk->scan & (kClkRcScans - 1)][blockIdx.x] = (unsigned long long)wall_clock64();
  }
}
__device__ __forceinline__ void rc_level0_body(int thread_num, const MP& mp, DevMap& m, int* __restrict__ next,
                                               int* __restrict__ sub, int* __restrict__ cand, int* __restrict__ rc,
                                               uint32_t* __restrict__ cand_bits, const WinD* __restrict__ win,
                                               uint64_t* __restrict__ ev, int* __restrict__ rcinfo, int cap);
// clk_end: this launch ends the scan's recut levels (max_layer 0)
__global__ void __launch_bounds__(64 * kRcFusedWaves) k_rc_level0(int thread_num, MP mp, DevMap m,
                                                                  int* __restrict__ next, int* __restrict__ sub,
                                                                  int* __restrict__ cand, int* __restrict__ rc,
                                                                  uint32_t* __restrict__ cand_bits,
                                                                  const WinD* __restrict__ win,
                                                                  uint64_t* __restrict__ ev,
                                                                  int* __restrict__ rcinfo, int cap, KClock* clk,
                                                                  int clk_end) {
  rc_clock_start(clk);
  rc_level0_body(thread_num, mp, m, next, sub, cand, rc, cand_bits, win, ev, rcinfo, cap);
  if (clk_end) rc_clock_end(clk);
}
__device__ __forceinline__ void rc_level0_body(int thread_num, const MP& mp, DevMap& m, int* __restrict__ next,
                                               int* __restrict__ sub, int* __restrict__ cand, int* __restrict__ rc,
                                               uint32_t* __restrict__ cand_bits, const WinD* __restrict__ win,
                                               uint64_t* __restrict__ ev, int* __restrict__ rcinfo, int cap) {
  if (blockIdx.x == 0 && threadIdx.x == 0) rc[kRcNode0] = m.counters[kCntNodes];  // k_rc_level(0)'s id base
  if (rc[kRcAbort]) return;
  if (g_slide(m) < thread_num) return;  // local_mapping.cpp:150-154 (global count)
  const int nw = m.counters[kCntSlide];
  const bool wide = win->win_count > 63;
  if (wide && mp.max_layer > 0) {
    if (threadIdx.x == 0 && blockIdx.x == 0) atomicOr(&m.counters[kCntErr], 16);
  }
  const bool do_win = mp.max_layer > 0 && !wide;
  const int nwv = gridDim.x * kRcFusedWaves;
  for (int j = blockIdx.x * kRcFusedWaves + (threadIdx.x >> 6); j * 64 < nw; j += nwv)
    rc_visit_chunk(0, m.slide, nw, j, mp, m, next, sub, cand, rc, cand_bits, do_win, win, ev, rcinfo, cap);
}

__device__ __forceinline__ void rc_level_body(
    int L, int sub_cap, const MP& mp, DevMap& m, const int* __restrict__ sub_in, const int* __restrict__ info_in,
    const uint64_t* __restrict__ ev_in, int* __restrict__ next, int* __restrict__ next2, int* __restrict__ sub_out,
    int* __restrict__ cand, int* __restrict__ rc, uint32_t* __restrict__ cand_bits, const WinD* __restrict__ win,
    uint64_t* __restrict__ ev_out, int* __restrict__ info_out, int cap);
// clk_end: the scan's last level kernel (its workgroups stamp the recut's end)
__global__ void __launch_bounds__(64 * kRcFusedWaves) k_rc_level(
    int L, int sub_cap, MP mp, DevMap m, const int* __restrict__ sub_in, const int* __restrict__ info_in,
    const uint64_t* __restrict__ ev_in, int* __restrict__ next, int* __restrict__ next2, int* __restrict__ sub_out,
    int* __restrict__ cand, int* __restrict__ rc, uint32_t* __restrict__ cand_bits, const WinD* __restrict__ win,
    uint64_t* __restrict__ ev_out, int* __restrict__ info_out, int cap, KClock* clk, int clk_end) {
  rc_level_body(L, sub_cap, mp, m, sub_in, info_in, ev_in, next, next2, sub_out, cand, rc, cand_bits, win, ev_out,
                info_out, cap);
  if (clk_end) rc_clock_end(clk);
}
__device__ __forceinline__ void rc_level_body(
    int L, int sub_cap, const MP& mp, DevMap& m, const int* __restrict__ sub_in, const int* __restrict__ info_in,
    const uint64_t* __restrict__ ev_in, int* __restrict__ next, int* __restrict__ next2, int* __restrict__ sub_out,
    int* __restrict__ cand, int* __restrict__ rc, uint32_t* __restrict__ cand_bits, const WinD* __restrict__ win,
    uint64_t* __restrict__ ev_out, int* __restrict__ info_out, int cap) {
  __shared__ __attribute__((aligned(16))) int s_in[kApplySub];
  __shared__ int s_sub[kApplySub], s_q[kApplySub], s_mask[kApplySub], s_coff[kApplySub];
  __shared__ int s_ws[kRcFusedWaves];
  __shared__ double E[kRcFusedWaves][64][kErec];
  __shared__ int s_slot[kRcFusedWaves][64];
  __shared__ double s_pre[kRcFusedWaves][32 * 10];
  if (rc[kRcAbort]) return;
  const int nsub = rc[kRcSub + L];
  if (nsub > sub_cap) {  // the host-sized path replays from this level
    if (blockIdx.x == 0 && threadIdx.x == 0) rc[kRcAbort] = L + 1;
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ntot = rc[kRcNch + L];  // children of this level's subdividing leaves (rc_win_leaf)
  const int A = rc[kRcLvl + L];     // level L+1's other nodes (visit(L))
#ifdef VG_PROBE
  const int pb = L < 2 ? 8 * L : 32;  // per level: calls, sort, prefix, push, tail, nsub, ntot, A (block 0)
  VG_PROBE_BEGIN();
  if (blockIdx.x == 0 && tid == 0 && L < 3) {
    atomicAdd(&g_probe[pb], 1ull);
    atomicAdd(&g_probe[pb + 5], (unsigned long long)nsub);
    atomicAdd(&g_probe[pb + 6], (unsigned long long)ntot);
    atomicAdd(&g_probe[pb + 7], (unsigned long long)A);
  }
#define RC_MARK(k) \
  do {             \
    if (blockIdx.x == 0 && L < 3) VG_PROBE_MARK(pb + (k)); \
  } while (0)
#else
#define RC_MARK(k) (void)0
#endif
  const int base = (L == 0) ? rc[kRcNode0] : rc[kRcChBase + L - 1] + rc[kRcCh + L - 1];
  if (blockIdx.x == 0 && tid == 0) {
    rc[kRcCh + L] = ntot;
    rc[kRcChBase + L] = base;
    rc[kRcTot + L] = A + ntot;
    m.counters[kCntNodes] = base + ntot;
  }
  const bool wide = win->win_count > 63;
  const bool do_win = (L + 1 < mp.max_layer) && !wide;
  if (wide && L + 1 < mp.max_layer && blockIdx.x == 0 && tid == 0) atomicOr(&m.counters[kCntErr], 16);
  // every subdividing leaf becomes internal (alloc_parent's mark, sub_finish), children or not; the
  // pushes below read only the parents' fix_off and geometry, which this leaves alone
  for (int i = blockIdx.x * blockDim.x + tid; i < nsub; i += gridDim.x * blockDim.x) {
    const int p = sub_in[i];
    m.nscr[(size_t)p * 4 + 1] = -1;
    sub_finish(m, p);
  }
  if ((int)blockIdx.x * kRcFusedWaves < ntot) {
    // apply(L): the subdividing leaves in ascending id order (rank among distinct ids, from LDS),
    // each with its rcinfo slot (its index in sub_in, rc_win_leaf's q) and octant mask, read in
    // the same round as the ids
    constexpr int kPer = kApplySub / (64 * kRcFusedWaves);
    int mk_t[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const int t = tid + k * 64 * kRcFusedWaves;
      s_in[t] = t < nsub ? sub_in[t] : 0x7fffffff;
      mk_t[k] = (t < nsub && (size_t)t * kRcInfo + kRcInfo <= (size_t)cap) ? info_in[(size_t)t * kRcInfo + 17] : 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const int t = tid + k * 64 * kRcFusedWaves;
      if (t >= nsub) break;
      const int myp = s_in[t];
      int rank = 0;
      const int4* v4 = reinterpret_cast<const int4*>(s_in);
      for (int u = 0; u < (nsub + 3) / 4; u++) {
        const int4 v = v4[u];
        rank += (v.x < myp) + (v.y < myp) + (v.z < myp) + (v.w < myp);
      }
      s_sub[rank] = myp;
      s_q[rank] = t;
      s_mask[rank] = mk_t[k];
    }
    __syncthreads();
    RC_MARK(1);
    // per parent: its rcinfo slot and non-empty octants; exclusive prefix of their counts (4 per thread)
    int c4[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int t = 4 * tid + k;
      c4[k] = 0;
      if (t < nsub) c4[k] = __popc(s_mask[t]);
      sum += c4[k];
    }
    int x = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) s_ws[wv] = x;
    __syncthreads();
    int run = x - sum;
    for (int k = 0; k < wv; k++) run += s_ws[k];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int t = 4 * tid + k;
      if (t < nsub) s_coff[t] = run;
      run += c4[k];
    }
    __syncthreads();
    RC_MARK(2);
    const RoleIdx ri0 = rc_push_role(lane), ri1 = rc_push_role(lane + 64 < 72 ? lane + 64 : 0);
    for (int c = blockIdx.x * kRcFusedWaves + wv; c < ntot; c += gridDim.x * kRcFusedWaves) {
      int lo = 0, hi = nsub - 1;  // the parent: the last t with s_coff[t] <= c
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_coff[mid] <= c) lo = mid;
        else hi = mid - 1;
      }
      const int t = lo, p = s_sub[t], k = c - s_coff[t];
      int mk = s_mask[t];
      for (int i = 0; i < k; i++) mk &= mk - 1;
      const int o = __ffs(mk) - 1;  // the parent's k-th non-empty octant
      if (o < 0) continue;
#ifdef VG_PROBE
      unsigned long long qt = wall_clock64();  // workgroup 0's wave 0: 48 init, 49 push, 51 visit, 52 win, 53 wins
      const bool qpr = blockIdx.x == 0 && tid == 0;
#define Q_MARK(k)                                   \
  do {                                              \
    if (qpr) {                                      \
      const unsigned long long n_ = wall_clock64(); \
      atomicAdd(&g_probe[(k)], n_ - qt);            \
      qt = n_;                                      \
    }                                               \
  } while (0)
#else
#define Q_MARK(k) (void)0
#endif
      const int* inf = info_in + (size_t)s_q[t] * kRcInfo;
      const int j0 = inf[0] + inf[1 + o], j1 = j0 + inf[9 + o];
      const int child = base + c;
      if (child >= m.cap_nodes) {
        if (lane == 0) atomicOr(&m.counters[kCntErr], 4);
        continue;
      }
      NodeHdr& ph = m.hdr[p];
      const int layer = ph.layer + 1;
      if (lane == 0) {  // alloc_parent for this octant
        const int xyz[3] = {(o >> 2) & 1, (o >> 1) & 1, o & 1};
        double cc[3];
        for (int jj = 0; jj < 3; jj++) cc[jj] = ph.center[jj] + (float)((2 * xyz[jj] - 1) * ph.qlen);
        init_node(m.hdr[child], cc, ph.qlen / 2, layer, p);
        dbox_child(m.dbox + (size_t)child * 6, m.dbox + (size_t)p * 6, ph.center, o);
        ph.child[o] = child;
        m.cfirst[(size_t)p * 8 + o] = 0x7f7f7f7f;
        next[A + c] = child;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      Q_MARK(48);
      rc_push_child(child, p, layer, j0, j1, ev_in, mp, win, m, E[wv], s_slot[wv], s_pre[wv], ri0, ri1);
      Q_MARK(49);
      // visit(L+1) of the new child (its cluster, counts and flags: this wave's stores just above)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      int kids[8], nchild, is_cand, is_sub;
      recut_visit_node(lane == 0 ? child : -1, mp, m, kids, nchild, is_cand, is_sub);
      int o1, o2, o3;
      wave_append3(&rc[kRcLvl + L + 1], 0, &m.counters[kCntFactors], is_cand, &rc[kRcSub + L + 1], is_sub, o1, o2,
                   o3);
      if (is_cand) {
        cand[o2] = child;
        if (cand_bits) atomicOr(&cand_bits[child >> 5], 1u << (child & 31));
      }
      if (is_sub) sub_out[o3] = child;
      Q_MARK(51);
      if (do_win && __shfl(is_sub, 0, 64)) {
        rc_win_leaf(L + 1, child, __shfl(o3, 0, 64), win, m, ev_out, info_out, cap, cap, rc);
#ifdef VG_PROBE
        if (qpr) atomicAdd(&g_probe[53], 1ull);
#endif
      }
      Q_MARK(52);
#undef Q_MARK
    }
    RC_MARK(3);
  }
  // visit(L+1) (+ win(L+1)) of the level's other nodes, from the grid's last waves
  const int nwv = gridDim.x * kRcFusedWaves;
  for (int j = nwv - 1 - ((int)blockIdx.x * kRcFusedWaves + wv); j * 64 < A; j += nwv)
    rc_visit_chunk(L + 1, next, A, j, mp, m, next2, sub_out, cand, rc, cand_bits, do_win, win, ev_out, info_out, cap);
  RC_MARK(4);
#undef RC_MARK
}

// ---- host-sized path (overflow replay) ----------------------------------
// the children's event ranges of the sorted parents (ids c0 + prefix, as
// alloc_children handed them out)
__global__ void __launch_bounds__(256) k_sub_cseg(int ns, const int* __restrict__ sub, const uint32_t* __restrict__ off,
                                                  DevMap m, const int* __restrict__ rcinfo, int* __restrict__ cseg) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ns; q += gridDim.x * blockDim.x)
    rc_child_segs(m, sub[q], (int)off[q], rcinfo, cseg);
}
__global__ void __launch_bounds__(256) k_sub_finish(int ns, const int* __restrict__ sub, DevMap m) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ns; q += gridDim.x * blockDim.x) sub_finish(m, sub[q]);
}

// tras_opt: factor list in node-id order; opt_state = factor index
__global__ void __launch_bounds__(256) k_factor_finish(int nf, const int* __restrict__ fac, DevMap m, int* __restrict__ fac_node,
                                double* __restrict__ fac_eig, Clu* __restrict__ fac_pcr) {
  for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < nf; a += gridDim.x * blockDim.x) {
    int node = fac[a];
    fac_node[a] = node;
    m.hdr[node].opt_state = a;
    for (int j = 0; j < 12; j++) fac_eig[(size_t)a * 12 + j] = m.eig[(size_t)node * 12 + j];
    fac_pcr[a] = m.pcr_add[node];
  }
}

// a recut level's subdividing leaves, rcinfo and events (alternate buffers per level)
static int* sub_of(Work& w, int L) { return (L % 2 == 0) ? w.list2 : w.sub_odd; }
static int* info_of(Work& w, int L) { return (L % 2 == 0) ? (int*)w.v1 : w.info_odd; }
static uint64_t* ev_of(Work& w, int L) { return (L % 2 == 0) ? w.k0 : w.ev_odd; }

static int read_rc(vg_ctx* ctx, int* h) {
  VG_HIP(hipMemcpyAsync(h, ctx->wk.rc, kRcN * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  return read_counters(ctx);  // synchronizes
}

// host-sized apply of level L (k_rc_visit and k_rc_win already ran): sorted
// subdividing leaves, host-sized child allocation, the children's event
// ranges, then the device pushes (k_rc_push) and the parents' finish
static int recut_slow_apply(vg_ctx* ctx, int L, const MP& mp, WinD* dwin, int* next, int* hrc) {
  DevMap& m = ctx->map;
  Work& w = ctx->wk;
  hipStream_t s = ctx->stream;
  const int nsub = hrc[kRcSub + L], nnext = hrc[kRcLvl + L];
  if (nsub <= 0) return VG_OK;
  int* sub = sub_of(w, L);
  VG_TRY(sort_ids_inplace(ctx, sub, nsub));
  VG_TRY(read_counters(ctx));
  const int first = ctx->h_pinned[kCntNodes];
  int created = 0;
  VG_TRY(alloc_children(ctx, sub, nsub, next, nnext, true, &created));
  k_sub_cseg<<<grid_for(nsub), kBlock, 0, s>>>(nsub, sub, w.ac_off, m, info_of(w, L), (int*)w.ac_cnt);
  VG_HIP(hipMemsetD32Async((hipDeviceptr_t)(w.rc + kRcLvl + L), nnext + created, 1, s));
  VG_HIP(hipMemsetD32Async((hipDeviceptr_t)(w.rc + kRcCh + L), created, 1, s));
  VG_HIP(hipMemsetD32Async((hipDeviceptr_t)(w.rc + kRcChBase + L), first, 1, s));
  k_rc_push<<<256, 64 * kRcPushWaves, 0, s>>>(L, ev_of(w, L), (const int*)w.ac_cnt, mp, dwin, m, w.rc);
  k_sub_finish<<<grid_for(nsub), kBlock, 0, s>>>(nsub, sub, m);
  VG_HIP(hipGetLastError());
  return read_counters(ctx);
}

// recut start: zero the level counts and the factor count; an insert whose
// child allocation overflowed (kCntMisc) blocks the whole recut (rc abort code
// kInsAbort) until map_insert_replay has run
constexpr int kInsAbort = 100;
__device__ __forceinline__ void recut_begin_block(DevMap& m, int* __restrict__ rc, int thread_num) {
  const int t = threadIdx.x;
  for (int i = t; i < kRcN; i += blockDim.x) rc[i] = 0;
  __syncthreads();
  if (t == 0) {
    m.counters[kCntFactors] = 0;
    m.counters[kCntGSlide] = m.counters[kCntSlide];  // all-reduced next in sharded mode
    if (m.counters[kCntMisc] != 0 && g_touched(m) >= thread_num) rc[kRcAbort] = kInsAbort;
  }
}
// the recut's head as one launch: the window view (poses from the device
// state, ring, per-ord counts), then the level counters cleared
__global__ void k_make_win_recut_begin(DState* __restrict__ st, WinArg wa, const int* __restrict__ wpn,
                                       WinD* __restrict__ win, int* __restrict__ nper, int* __restrict__ slot_of,
                                       DevMap m, int* __restrict__ rc, int thread_num) {
  make_win_block(st, wa, wpn, win, nper, slot_of);
  __syncthreads();
  recut_begin_block(m, rc, thread_num);
}

// Asynchronous factor extraction (tras_opt, octree.cpp:491-516) sized on the
// device. k_rc_visit marks every candidate in a bitmap over node ids; one
// workgroup turns the bitmap into the id-ascending factor list (the host
// path's sort order) with one prefix sum over the allocated id range, clearing
// it as it reads, then k_factor_finish_dev fills the factor arrays. k_fac_sort
// also publishes the recut status and the factor count (Pub::seq_rc) and
// leaves the status in rc[kRcStatus], where k_ba_init reads it: a recut that
// needs the host-sized path (insert replay, level overflow, more factors than
// max_fac) makes the LM skip, and the host completes the recut and reruns it.
// xa.frame (sharded): the status goes out in the exchange frame (site 5),
// closed here; k_pub_rc takes the sum
__global__ void __launch_bounds__(1024) k_fac_sort(DevMap m, int* __restrict__ rc, uint32_t* __restrict__ bits,
                                                   int* __restrict__ fac_node, int cap_f, Pub* __restrict__ pub,
                                                   int* __restrict__ seq_ctr, int max_fac, XchgArg xa) {
  fac_sort_block(m, rc, bits, fac_node, cap_f, pub, seq_ctr, max_fac, xa.frame == nullptr);
  if (xa.frame) {
    for (int i = threadIdx.x + 1; i < xa.n - 2; i += blockDim.x) xa.frame[i] = 0.0;
    if (threadIdx.x == 0) {  // (fac_sort_block's thread 0 wrote rc[kRcStatus])
      xa.frame[0] = (double)rc[kRcStatus];
      xchg_close(xa.frame, xa.n, 5, xa.seq);
    }
  }
}
// sharded mode: the recut status summed over the ranks into rc[kRcStatus], so
// every rank's k_ba_init skips alike and every host takes the same host-sized
// completion and LM rerun — the ranks' exchange sequences stay in step (a
// guard mismatch: error bit 32, VG_E_STATE with the scan's counters). The
// factor count published is this rank's own.
__global__ void k_pub_rc(const DevMap m, int* __restrict__ rc, Pub* __restrict__ pub, const int* __restrict__ seq_ctr,
                         XchgArg xa) {
  if (threadIdx.x == 0) {
    const bool ok = xchg_ok(xa.frame, xa.n, xa.world);
    if (!ok) atomicOr(xa.err, 32);
    const int status = ok ? (int)llrint(xa.frame[0]) : 0;
    rc[kRcStatus] = status;
    pub_store(&pub->rc_status, status);
    pub_store(&pub->rc_nf, m.counters[kCntFactors]);
    pub_flag(&pub->seq_rc, *seq_ctr);
  }
}
__global__ void __launch_bounds__(256) k_factor_finish_dev(const int* __restrict__ rc, DevMap m,
                                                           const int* __restrict__ fac_node,
                                                           double* __restrict__ fac_eig, Clu* __restrict__ fac_pcr) {
  if (rc[kRcStatus]) return;
  const int nf = m.counters[kCntFactors];
  for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < nf; a += gridDim.x * blockDim.x) {
    const int node = fac_node[a];
    m.hdr[node].opt_state = a;
    for (int j = 0; j < 12; j++) fac_eig[(size_t)a * 12 + j] = m.eig[(size_t)node * 12 + j];
    fac_pcr[a] = m.pcr_add[node];
  }
}
const int* map_rc_status(vg_ctx* ctx) { return ctx->wk.rc + kRcStatus; }
// the factor bookkeeping an asynchronous recut left to a k_ba_init that did not come
int map_factor_finish(vg_ctx* ctx) {
  if (!ctx->rc_finish_in_init) return VG_OK;
  ctx->rc_finish_in_init = false;
  k_factor_finish_dev<<<64, 256, 0, ctx->stream>>>(ctx->wk.rc, ctx->map, ctx->ba.fac_node, ctx->ba.fac_eig,
                                                   ctx->ba.fac_pcr);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

// Test-only (vgx_memo_probe): the IEKF memo at centre planes. For every
// internal node, points exactly on its centre plane along each axis (the
// other two coordinates at +-hl/2) are looked up afresh (hash + descent, the
// reference's path: voxel_map.cpp:241-266, octree.cpp:586) and through the
// memo of the same point one ulp above / below the plane (the previous
// iteration's leaf). out: [0] samples, [1] memo != descent with the
// inclusive box (OctoTree::inside), [2] memo != descent with the descent's
// region (dbox, what k_iekf uses), [3] samples whose memo leaf differs from
// the fresh one (the plane really separates two leaves).
__global__ void __launch_bounds__(256) k_memo_probe(MP mp, DevMap m, int* __restrict__ out) {
  const int nn = m.counters[kCntNodes];
  int cnt[4] = {0, 0, 0, 0};
  for (int node = blockIdx.x * blockDim.x + threadIdx.x; node < nn; node += gridDim.x * blockDim.x) {
    const NodeHdr& h = m.hdr[node];
    if (h.octo != 1) continue;
    const double hl = h.qlen * 2;
    for (int j = 0; j < 3; j++)
      for (int sgn = 0; sgn < 4; sgn++)
        for (int side = 0; side < 2; side++) {
          V3 w = v3(h.center[0], h.center[1], h.center[2]);
          int k1 = (j + 1) % 3, k2 = (j + 2) % 3;
          w[k1] += ((sgn & 1) ? 0.5 : -0.5) * hl;
          w[k2] += ((sgn & 2) ? 0.5 : -0.5) * hl;
          V3 w2 = w;
          w2[j] = nextafter(w[j], side ? 1e300 : -1e300);
          uint64_t key, key2;
          if (!pack_key(w, mp.vs, key) || !pack_key(w2, mp.vs, key2) || key != key2) continue;
          const int root = hash_find(m.hkey, m.hval, m.hash_mask, key);
          if (root < 0) continue;
          const int fresh = descend(m.hdr, root, w), memo = descend(m.hdr, root, w2);
          if (fresh < 0 || memo < 0) continue;
          uint64_t kl;
          const NodeHdr& hm = m.hdr[memo];
          const bool same_root = pack_key(v3(hm.center[0], hm.center[1], hm.center[2]), mp.vs, kl) && kl == key;
          const int p_old = (same_root && inside(hm, w)) ? memo : fresh;
          const int p_new = (same_root && in_dbox(m.dbox + (size_t)memo * 6, w)) ? memo : fresh;
          cnt[0]++;
          cnt[1] += p_old != fresh;
          cnt[2] += p_new != fresh;
          cnt[3] += memo != fresh;
        }
  }
  for (int k = 0; k < 4; k++)
    if (cnt[k]) atomicAdd(&out[k], cnt[k]);
}
int map_memo_probe(vg_ctx* ctx, const MP& mp, int* out) {
  int* dout = reinterpret_cast<int*>(ctx->wk.partials);  // scratch: the probe runs between scans
  VG_HIP(hipMemsetAsync(dout, 0, 4 * sizeof(int), ctx->stream));
  k_memo_probe<<<256, 256, 0, ctx->stream>>>(mp, ctx->map, dout);
  VG_HIP(hipGetLastError());
  VG_HIP(hipMemcpyAsync(out, dout, 4 * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  VG_HIP(hipStreamSynchronize(ctx->stream));
  return VG_OK;
}
int map_set_attrs(vg_ctx* ctx) {
  (void)ctx;
  return VG_OK;
}

// the host-sized rest of a recut whose device status (hrc) is in: insert
// replay request, level-overflow replay, factor sort and extraction
static int recut_complete(vg_ctx* ctx, const MP& mp, int nlev, int* hrc, int* n_factors) {
  Work& w = ctx->wk;
  hipStream_t s = ctx->stream;
  DevMap& m = ctx->map;
  WinD* dwin = (WinD*)ctx->ba.xs;
  auto list_of = [&](int L) { return (L % 2 == 1) ? w.list0 : w.list1; };
  if (hrc[kRcAbort] == kInsAbort) return kNeedInsertReplay;
  if (hrc[kRcAbort]) {  // replay from the level that overflowed on the host-sized path
    const int L0 = hrc[kRcAbort] - 1;
#ifdef VG_PROBE
    fprintf(stderr, "PROBE recut overflow replay from level %d (nsub=%d nwin=%d)\n", L0, hrc[kRcSub + L0],
            hrc[kRcWin + L0]);
#endif
    VG_HIP(hipMemsetAsync(w.rc + kRcAbort, 0, sizeof(int), s));
    VG_TRY(recut_slow_apply(ctx, L0, mp, dwin, list_of(L0 + 1), hrc));
    int* dn = (int*)((char*)ctx->ba.xs + sizeof(WinD));
    int* dslot = dn + 32;
    const int total = ctx->rc_total;
    for (int L = L0 + 1; L < nlev; L++) {
      k_rc_visit<<<256 * kBlock / kSpreadBlock, kSpreadBlock, 0, s>>>(L, ctx->rc_thread_num, list_of(L), mp, m, list_of(L + 1), sub_of(w, L), w.cand,
                                        w.rc, nullptr);
      k_rc_win<<<256, 64 * kRcWinWaves, 0, s>>>(L, sub_of(w, L), dwin, m, ev_of(w, L), info_of(w, L), w.cap, w.cap, w.rc);
      VG_TRY(read_rc(ctx, hrc));
      VG_TRY(recut_slow_apply(ctx, L, mp, dwin, list_of(L + 1), hrc));
    }
  }
  VG_HIP(hipMemsetAsync(w.rc + kRcStatus, 0, sizeof(int), s));  // the LM rerun reads it
  VG_TRY(read_counters(ctx));
  const int nf = ctx->h_pinned[kCntFactors];
  if (nf > ctx->ba.cap_f) {
    ctx->err = "factor capacity exceeded";
    return VG_E_CAPACITY;
  }
  if (nf > 0) {
    int* sorted = w.cand;
    VG_TRY(sort_ids(ctx, w.cand, nf, &sorted));
    k_factor_finish<<<grid_for(nf), kBlock, 0, s>>>(nf, sorted, m, ctx->ba.fac_node, ctx->ba.fac_eig,
                                                    ctx->ba.fac_pcr);
    VG_HIP(hipGetLastError());
  }
  *n_factors = nf;
  return VG_OK;
}

// multi_recut (local_mapping.cpp:144-201) then tras_opt. Synchronous
// (pub_seq == 0): returns the factor count, or kNeedInsertReplay when the
// preceding insert must be replayed first (nothing of the recut ran).
// Asynchronous (pub_seq > 0): the factor extraction is sized on the device and
// nothing waits; *n_factors = -1 and the status arrives with Pub::seq_rc ==
// pub_seq (map_recut_resume completes a recut that needs the host).
static int map_recut_impl(vg_ctx* ctx, const MP& mp, const WinArg& wa, int thread_num, int* n_factors, bool replay,
                          int pub_seq) {
  DevMap& m = ctx->map;
  Work& w = ctx->wk;
  hipStream_t s = ctx->stream;
  *n_factors = 0;
  // the window view (poses from the device state, ring, per-ord counts)
  WinD* dwin = (WinD*)ctx->ba.xs;
  int* dn = (int*)((char*)ctx->ba.xs + sizeof(WinD));
  int* dslot = dn + 32;
  int total = 0;
  for (int i = 0; i < wa.win_count; i++) total += wa.nper[i];
  ctx->rc_total = total;
  ctx->rc_thread_num = thread_num;
  if (ctx->rc_begun) {  // done by the insert's k_push_window (the same graph)
    ctx->rc_begun = false;
  } else {
    k_make_win_recut_begin<<<1, 256, 0, s>>>(ctx->st, wa, ctx->map.wpn, dwin, dn, dslot, m, w.rc, thread_num);
  }
  if (sharded(ctx)) {
    if (!replay) {  // the global slide count (a replay re-uses it: the insert replay does not change it)
      VG_TRY(shard_allreduce(ctx, m.counters + kCntGSlide, ctx->shard.d_buf + 512, 1, 1, 2));
    }
    k_copy_int<<<1, 64, 0, s>>>((const int*)(ctx->shard.d_buf + 512), m.counters + kCntGSlide);
  }
  const int nlev = mp.max_layer + 1;  // children sit one layer down; leaves at max_layer do not subdivide
  auto list_of = [&](int L) { return (L % 2 == 1) ? w.list0 : w.list1; };  // worklist of level L >= 1
  constexpr int gv = 256;
  const int gw = grid_for(total > 0 ? total : 1, kBlock, 2048);  // grid-stride over the device total
  const int sub_cap = (ctx->dbg_apply_cap >= 0 && ctx->dbg_apply_cap < kApplySub) ? ctx->dbg_apply_cap : kApplySub;
  uint32_t* bits = pub_seq > 0 ? w.cand_bits : nullptr;
  if (ctx->rc_fused) {  // one launch per level boundary (k_rc_level0, k_rc_level)
    static_assert(gv <= kClkRcBlocks, "recut clock slots");
    k_rc_level0<<<gv, 64 * kRcFusedWaves, 0, s>>>(thread_num, mp, m, list_of(1), sub_of(w, 0), w.cand, w.rc, bits,
                                                 dwin, ev_of(w, 0), info_of(w, 0), w.cap, &ctx->st->clk,
                                                 mp.max_layer == 0 ? 1 : 0);
    for (int L = 0; L < mp.max_layer; L++)
      k_rc_level<<<gv, 64 * kRcFusedWaves, 0, s>>>(L, sub_cap, mp, m, sub_of(w, L), info_of(w, L), ev_of(w, L),
                                                  list_of(L + 1), list_of(L + 2), sub_of(w, L + 1), w.cand, w.rc,
                                                  bits, dwin, ev_of(w, L + 1), info_of(w, L + 1), w.cap, &ctx->st->clk,
                                                  L == mp.max_layer - 1 ? 1 : 0);
  } else {
    for (int L = 0; L < nlev; L++) {
      k_rc_visit<<<gv * kBlock / kSpreadBlock, kSpreadBlock, 0, s>>>(L, thread_num, L > 0 ? list_of(L) : nullptr, mp, m,
                                                                     list_of(L + 1), sub_of(w, L), w.cand, w.rc, bits);
      // nodes at layer max_layer never subdivide (recut_visit_node, octree.cpp:371-372):
      // the deepest level has no window events, no apply and no pushes
      if (L == mp.max_layer) break;
      k_rc_win<<<256, 64 * kRcWinWaves, 0, s>>>(L, sub_of(w, L), dwin, m, ev_of(w, L), info_of(w, L), w.cap, w.cap,
                                                w.rc);
      k_rc_apply<<<1, kApplyThreads, 0, s>>>(L, sub_cap, m, list_of(L + 1), sub_of(w, L), info_of(w, L),
                                             (int*)w.ac_off, w.rc);
      k_rc_push<<<64, 64 * kRcPushWaves, 0, s>>>(L, ev_of(w, L), (const int*)w.ac_off, mp, dwin, m, w.rc);
    }
  }
  VG_HIP(hipGetLastError());
  if (pub_seq > 0) {
    const int max_fac = (ctx->dbg_fac_max >= 0 && ctx->dbg_fac_max < kFacMax) ? ctx->dbg_fac_max : kFacMax;
    const bool shard_on = sharded(ctx);
    Shard& sh = ctx->shard;
    const XchgArg xa{shard_on ? sh.d_frame : nullptr, sh.d_seq, m.counters + kCntErr, kShardSmall, sh.world};
    k_fac_sort<<<1, 1024, 0, s>>>(m, w.rc, w.cand_bits, ctx->ba.fac_node, ctx->ba.cap_f, ctx->d_pub,
                                  &ctx->st->rc_ctr, max_fac, xa);
    if (shard_on) {
      VG_TRY(shard_exchange(ctx, kShardSmall));
      k_pub_rc<<<1, 64, 0, s>>>(m, w.rc, ctx->d_pub, &ctx->st->rc_ctr, xa);
    }
    if (ctx->rc_init_finish) {  // the LM's k_ba_init (next on the stream) does tras_opt's bookkeeping
      ctx->rc_finish_in_init = true;
    } else {
      k_factor_finish_dev<<<64, 256, 0, s>>>(w.rc, m, ctx->ba.fac_node, ctx->ba.fac_eig, ctx->ba.fac_pcr);
    }
    VG_HIP(hipGetLastError());
    *n_factors = -1;
    return VG_OK;
  }
  int* hrc = ctx->h_pinned + 128;
  VG_TRY(read_rc(ctx, hrc));
  return recut_complete(ctx, mp, nlev, hrc, n_factors);
}

// complete an asynchronous recut whose published status was nonzero (the LM
// skipped): same outcomes as the synchronous call
static int map_recut_resume_impl(vg_ctx* ctx, const MP& mp, int* n_factors) {
  int* hrc = ctx->h_pinned + 128;
  VG_TRY(read_rc(ctx, hrc));
  return recut_complete(ctx, mp, mp.max_layer + 1, hrc, n_factors);
}

// the recut's end on the main stream: the margi prefix (second stream) starts
// from it, under the LM iterations enqueued behind it
int map_recut(vg_ctx* ctx, const MP& mp, const WinArg& wa, int thread_num, int* n_factors, bool replay,
              int pub_seq) {
  const int r = map_recut_impl(ctx, mp, wa, thread_num, n_factors, replay, pub_seq);
  if (!ctx->capturing) VG_HIP(hipEventRecord(ctx->ev_recut_done, ctx->stream));  // else after the graph launch
  return r;
}
int map_recut_resume(vg_ctx* ctx, const MP& mp, int* n_factors) {
  const int r = map_recut_resume_impl(ctx, mp, n_factors);
  VG_HIP(hipEventRecord(ctx->ev_recut_done, ctx->stream));
  return r;
}

// ------------------------------------------------------------------ margi (A10)
// collect every node under the slide roots, level by level (top-down)
// level L of the surf_map_slide subtrees: level 0 is m.slide itself, levels
// >= 1 sit back to back in `lists` (level L at the sum of the counts of levels
// 1..L-1; the count of level L+1 is rc[L], appended by level L)
__device__ __forceinline__ int margi_level(int L, const DevMap& m, const int* rc, int* lists, int** work) {
  if (L == 0) {
    *work = m.slide;
    return m.counters[kCntSlide];
  }
  int off = 0;
  for (int l = 1; l < L; l++) off += rc[l - 1];
  *work = lists + off;
  return rc[L - 1];
}

// OctoTree::margi's bottom-up isexist (octree.cpp:485-494) without a launch
// per level: a node whose isexist is final reports it to its parent with one
// 64-bit atomic (children still to report in the high word, minus one; the
// existing ones in the low word, plus its bit); the child that reports last
// has every sibling's bit in the returned word, so it sets the parent's
// isexist = OR(children) and reports for the parent in turn. The payload is
// the atomic itself: no fence. Roots (parent -1) end the chain.
__device__ __forceinline__ void margi_exist_up(DevMap& m, int node, int ex) {
  for (int hop = 0; hop < 16; hop++) {
    const int par = m.hdr[node].parent;
    if (par < 0) return;
    const unsigned long long old = atomicAdd(&m.pend[par], (unsigned long long)ex - (1ull << 32));
    if ((old >> 32) != 1ull) return;  // a sibling reports later
    ex = ((unsigned)(old & 0xffffffffull) + (unsigned)ex) > 0u ? 1 : 0;
    m.hdr[par].isexist = (int8_t)ex;
    node = par;
  }
}

__global__ void __launch_bounds__(256) k_collect_level(int L, int thread_num, DevMap m, int* __restrict__ lists,
                                                       int* __restrict__ leaves, int* __restrict__ rc) {
  if (g_slide(m) < thread_num) return;
  int* work;
  const int nw = margi_level(L, m, rc, lists, &work);
  int* next;
  (void)margi_level(L + 1, m, rc, lists, &next);  // its count is still being appended
  const int next_off = (int)(next - lists);
  for (int base = blockIdx.x * blockDim.x; base < nw; base += gridDim.x * blockDim.x) {
    const int q = base + threadIdx.x;
    const int node = q < nw ? work[q] : -1;
    int nchild = 0, is_leaf = 0;
    int kids[8];
    if (node >= 0) {
      NodeHdr& h = m.hdr[node];
      if (h.octo == 1) {
        for (int o = 0; o < 8; o++)
          if (h.child[o] >= 0) kids[nchild++] = h.child[o];
        m.pend[node] = (unsigned long long)nchild << 32;  // margi_exist_up: children still to report
        if (nchild == 0) {  // internal_exist of a childless node: 0, reported now
          h.isexist = 0;
          margi_exist_up(m, node, 0);
        }
      } else {
        is_leaf = 1;
      }
    }
    int o1 = wave_append(&rc[L], nchild);
    int o2 = wave_append(&m.counters[kCntLeaves], is_leaf);
    if (next_off + o1 + nchild > m.cap_nodes) {
      atomicOr(&m.counters[kCntErr], 4);
      continue;
    }
    for (int j = 0; j < nchild; j++) next[o1 + j] = kids[j];
    if (is_leaf) leaves[o2] = node;
  }
}

__device__ void plane_update_dev(DevMap& m, int node, const Clu& pcr_add, const double* e) {
  PlaneRec& P = m.pl[node];
  V3 center = v3(pcr_add.v[0] / pcr_add.N, pcr_add.v[1] / pcr_add.N, pcr_add.v[2] / pcr_add.N);
  V3 u[3];
  for (int k = 0; k < 3; k++) u[k] = v3(e[3 + 0 * 3 + k], e[3 + 1 * 3 + k], e[3 + 2 * 3 + k]);
  double nv = 1.0 / pcr_add.N;
  M<3, 9> uc;
  uc.zero();
  const int l = 0;
  for (int k = 1; k < 3; k++) {
    M3 ukl = outer3(u[k], u[l]);
    double f[9];
    f[0] = ukl(0, 0);
    f[1] = ukl(1, 0) + ukl(0, 1);
    f[2] = ukl(2, 0) + ukl(0, 2);
    f[3] = ukl(1, 1);
    f[4] = ukl(1, 2) + ukl(2, 1);
    f[5] = ukl(2, 2);
    double a1 = dot3(u[k], center), a2 = dot3(u[l], center);
    for (int j = 0; j < 3; j++) f[6 + j] = -(u[l][j] * a1 + u[k][j] * a2);
    double sc = nv / (e[l] - e[k]);
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 9; c++) uc(r, c) += (u[k][r] * sc) * f[c];
  }
  M<9, 9> cov = unpack9(&m.cov_add[(size_t)node * kCovN]);
  M<3, 9> Jc = mul(uc, cov);
  M3 A = mul(Jc, tr(uc));
  double pv[6][6];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      pv[r][c] = A(r, c);
      pv[r][3 + c] = Jc(r, 6 + c) * nv;
      pv[3 + c][r] = pv[r][3 + c];
      pv[3 + r][3 + c] = cov(6 + r, 6 + c) * (nv * nv);
    }
  for (int r = 0; r < 6; r++)
    for (int c = r; c < 6; c++) P.var[sym_idx(6, r, c)] = pv[r][c];
  for (int j = 0; j < 3; j++) {
    P.center[j] = center[j];
    P.normal[j] = u[0][j];
  }
  P.radius = (float)e[2];
}

// OctoTree::margi leaf branch (octree.cpp:397-484), mgsize = 1. A leaf's
// run of the oldest slot (DevMap::lseg) is its sw->points[mp[0]] list in push
// order.
__global__ void __launch_bounds__(256) k_margi_leaf(const int* __restrict__ nleaves, const int* __restrict__ leaves,
                                                    MP mp, WinArg wa, DState* __restrict__ st, WinD* __restrict__ win,
                                                    int* __restrict__ nper, int* __restrict__ slot_of, int ba_iters_valid,
                                                    const int* __restrict__ ba_iters, const int* __restrict__ ba_hess,
                                                    Pub* __restrict__ pub, int seq, DevMap m,
                                                    const double* __restrict__ fac_eig, const Clu* __restrict__ fac_pcr,
                                                    int* __restrict__ plan, const int* __restrict__ gate,
                                                    unsigned* __restrict__ head_flag, int batch,
                                                    const int* __restrict__ dseq, const unsigned* __restrict__ pre_flag) {
  if (gate && !*gate) return;  // a speculative tail the LM did not reach (ba_run)
  if (pre_flag && blockIdx.x > 0) {  // the scan graph: the leaves read the margi prefix's lists (d_sync[4] >= ph[4])
    // Normally the prefix ended long before (it runs under the LM): its
    // writes were released at its end and this kernel's start acquired them,
    // so no fence. Only a workgroup that had to wait acquires after the wait
    // (an agent-scope acquire per workgroup invalidates the XCD's L2: with
    // ~2k workgroups that cost the kernel 14 us when every one did it)
    __shared__ int s_state;  // 0 ready at once, 1 waited, 2 timed out
    if (threadIdx.x == 0) {
      const unsigned t = (unsigned)st->ph[4];
      int state = 0;
      for (long it = 0; (int)(__hip_atomic_load(pre_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - t) < 0; it++) {
        state = 1;
        __builtin_amdgcn_s_sleep(4);
        if (it > (1l << 24)) {
          state = 2;
          atomicOr(&m.counters[kCntErr], 64);
          break;
        }
      }
      s_state = state;
    }
    __syncthreads();
    if (s_state == 2) return;
    if (s_state == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  if (blockIdx.x == 0) {  // the margi head: x_curr <- x_buf.back(), the window view, the state publication
    if (dseq) {  // the scan graph: this scan's publication numbers from the device state (DState::ph)
      seq = dseq[0];
      wa.seq2 = dseq[1];
      wa.jour_check = dseq[4];
    }
    make_win_block(st, wa, m.wpn, win, nper, slot_of);
    __syncthreads();  // x_curr (set_xc), seen by the whole block
    if (threadIdx.x == 0) st->margi_seq = seq;  // k_margi_copy hands it to the next IEKF
    // x_curr is final: the next scan's propagation may start (vg_ctx::d_sync[2]) as soon as
    // the publication has read what that propagation overwrites
    publish_state_block(st, wa.win_count, ba_iters_valid, ba_iters, ba_hess, pub, seq, head_flag, (unsigned)seq);
    return;
  }
  // the leaves read the refined window poses from the state (the view block
  // above writes the same values into *win for the later margi kernels)
  const double* xs = st->xs;
  const int nl = *nleaves;
#ifdef VG_PROBE
  const unsigned long long pt0 = wall_clock64();
  const bool pwork = (int)((blockIdx.x - 1) * blockDim.x) < nl;
#endif
  int n_pu = 0, n_full = 0;  // plane_update calls / leaves past max_points (per-scan counters)
#ifdef VG_PROBE
  // per leaf thread, summed over the live leaves (scripts/probe_margi.py): 51 header + run + own
  // cluster, 52 frame clusters + merge + eigen, 54 plane update, 55 point_fix carve + stores;
  // 56 live leaves, 57 the longest leaf, 58 factor leaves
  unsigned long long pq0 = wall_clock64(), pa = 0, pb2 = 0, pc = 0, pd = 0, ptot = 0, nlive = 0, nfac = 0;
#define PMG(v)                                   \
  do {                                           \
    const unsigned long long n_ = wall_clock64(); \
    v += n_ - pq0;                               \
    pq0 = n_;                                    \
  } while (0)
#else
#define PMG(v) (void)0
#endif
  // whole waves per round: the point_fix blocks that grow are carved with one
  // atomic per wave (wave_append) instead of one per leaf on the shared counter
  for (int base = (blockIdx.x - 1) * blockDim.x; base < nl; base += (gridDim.x - 1) * blockDim.x) {
    const int q = base + threadIdx.x;
    const int node = q < nl ? leaves[q] : -1;
    int* pq = &plan[(size_t)(q < nl ? q : 0) * 8];
    if (node >= 0) {
      pq[0] = -1;  // no point_fix copies (k_margi_copy)
      pq[4] = 0;
    }
    const bool live = node >= 0 && m.hdr[node].isexist && m.hdr[node].has_sw;
    const int W = mp.W;
    const int s0 = wa.mp[0];
#ifdef VG_PROBE
    const unsigned long long pstart = wall_clock64();
    pq0 = pstart;
#endif
    int seg = -1, segn = 0;  // the leaf's run of the oldest slot: its sw->points[mp[0]] in push order
    Clu w0, add_, fix_;
    int grow = 0;  // size of a new point_fix block (the live one is full)
    bool append = false;
    if (live) {
      NodeHdr& h = m.hdr[node];
      if (!lseg_get(m, node, s0, seg, segn)) seg = -1;
      Clu* loc = &m.pcrs[(size_t)node * W];
      const M3 R0 = ld_m3(xs);
      const V3 p0 = ld_v3(xs + 9);
      clu_zero(w0);
      if (loc[s0].N != 0) w0 = clu_transform(loc[s0], R0, p0);
      double* e = &m.eig[(size_t)node * 12];
      PMG(pa);
#ifdef VG_PROBE
      if (h.opt_state >= 0) nfac++;
#endif
      if (h.opt_state >= 0) {
        add_ = fac_pcr[h.opt_state];
        for (int j = 0; j < 12; j++) e[j] = fac_eig[(size_t)h.opt_state * 12 + j];
        h.opt_state = -1;
      } else {
        add_ = m.pcr_fix[node];
        if (batch) {  // the frame clusters read four at a time (one round trip each four), merged in frame order
          for (int i0 = 0; i0 < wa.win_count; i0 += 4) {
            Clu c[4];
#pragma unroll
            for (int k = 0; k < 4; k++)
              if (i0 + k < wa.win_count) c[k] = loc[wa.mp[i0 + k]];
#pragma unroll
            for (int k = 0; k < 4; k++) {
              const int i = i0 + k;
              if (i < wa.win_count && c[k].N != 0) {
                Clu t = (i == 0) ? w0 : clu_transform(c[k], ld_m3(xs + (size_t)i * kXS), ld_v3(xs + (size_t)i * kXS + 9));
                clu_add(add_, t);
              }
            }
          }
        } else {
          for (int i = 0; i < wa.win_count; i++) {
            int si = wa.mp[i];
            if (loc[si].N != 0) {
              Clu t = (i == 0) ? w0 : clu_transform(loc[si], ld_m3(xs + (size_t)i * kXS), ld_v3(xs + (size_t)i * kXS + 9));
              clu_add(add_, t);
            }
          }
        }
        if (h.is_plane) {
          V3 ev;
          M3 U;
          eig3(clu_cov(add_), ev, U);
          for (int j = 0; j < 3; j++) e[j] = ev[j];
          for (int j = 0; j < 9; j++) e[3 + j] = U[j];
        }
      }
      fix_ = m.pcr_fix[node];
      PMG(pb2);
      if (fix_.N < mp.max_points && h.is_plane)
        if (add_.N - h.last_num >= 5 || h.last_num <= 10) {
          plane_update_dev(m, node, add_, e);
          h.last_num = add_.N;
          n_pu++;
        }
      PMG(pc);
      if (fix_.N >= mp.max_points) n_full++;
      if (fix_.N < mp.max_points) {
        if (w0.N != 0) {
          clu_add(fix_, w0);
          if (seg >= 0 && segn > 0) {
            append = true;
            const int need = h.fix_cnt + segn;
            if (need > h.fix_cap) grow = need * 2 < 128 ? 128 : need * 2;
          }
        }
      } else {
        if (w0.N != 0) clu_sub(add_, w0);
        h.fix_cnt = 0;
      }
    }
    const int off = wave_append(&m.counters[kCntFix], grow);
    if (live) {
      NodeHdr& h = m.hdr[node];
      bool ok = true;
      if (append) {
        if (grow > 0) {  // grow the point_fix block (old block is abandoned)
          if (off + grow > m.cap_fix) {
            atomicOr(&m.counters[kCntErr], 8);
            ok = false;
          } else {
            pq[0] = h.fix_off;  // grow: move the live block first
            pq[1] = h.fix_cnt;
            pq[2] = off;
            h.fix_off = off;
            h.fix_cap = grow;
          }
        }
        if (ok) {
          pq[3] = seg;  // then append the oldest frame's points of this leaf
          pq[4] = segn;
          pq[5] = h.fix_off + h.fix_cnt;
          h.fix_cnt += segn;
        }
      }
      if (ok) {
        clu_zero(m.pcrs[(size_t)node * W + s0]);
        m.pcr_fix[node] = fix_;
        m.pcr_add[node] = add_;
        h.isexist = (fix_.N >= add_.N) ? 0 : 1;
      }
#ifdef VG_PROBE
      PMG(pd);
      const unsigned long long tl = wall_clock64() - pstart;
      ptot = tl > ptot ? tl : ptot;
      nlive++;
#endif
    }
  }
#undef PMG
#ifdef VG_PROBE
  {
    unsigned long long v[7] = {pa, pb2, pc, pd, nlive, nfac, ptot};
    for (int off = 32; off > 0; off >>= 1)
      for (int k = 0; k < 7; k++) {
        const unsigned long long o = __shfl_xor(v[k], off, 64);
        v[k] = k == 6 ? (o > v[k] ? o : v[k]) : v[k] + o;
      }
    if ((threadIdx.x & 63) == 0 && blockIdx.x > 0 && v[4] > 0) {  // working waves only (few atomics)
      atomicAdd(&g_probe[51], v[0]);
      atomicAdd(&g_probe[52], v[1]);
      atomicAdd(&g_probe[54], v[2]);
      atomicAdd(&g_probe[55], v[3]);
      atomicAdd(&g_probe[56], v[4]);
      atomicAdd(&g_probe[58], v[5]);
      atomicMax(&g_probe[57], v[6]);
    }
  }
#endif
  wave_append(&m.counters[kCntPlaneUpd], n_pu);
  wave_append(&m.counters[kCntFixFull], n_full);
#ifdef VG_PROBE
  __syncthreads();
  if (threadIdx.x == 0 && pwork) {  // per working block: summed span, longest span, count; leaves
    const unsigned long long pt1 = wall_clock64();
    atomicAdd(&g_probe[46], pt1 - pt0);
    atomicMax(&g_probe[45], pt1 - pt0);
    atomicAdd(&g_probe[47], 1ull);
    atomicMax(&g_probe[50], (unsigned long long)nl);
  }
#endif
}

// the point_fix copies planned by k_margi_leaf, one wave per leaf: the live
// block moves when it grows, then the leaf's points of the oldest frame are
// appended in push order (octree.cpp:450-458)
constexpr int kCopyWaves = 4;
// exist_up: the leaves also report their isexist up the tree (margi_exist_up,
// k_margi_erase_all follows); each leaf's report rides on a lane of its own
__global__ void __launch_bounds__(64 * kCopyWaves) k_margi_copy(const int* __restrict__ nleaves,
                                                                const int* __restrict__ plan,
                                                                const WinD* __restrict__ win, DevMap m, const int* __restrict__ gate,
                                                                const int* __restrict__ leaves, int exist_up,
                                                                unsigned* __restrict__ tail_flag,
                                                                const DState* __restrict__ st) {
  if (gate && !*gate) return;  // a speculative tail the LM did not reach (ba_run)
  // k_margi_leaf (the plane updates the next IEKF reads) has ended: its writes
  // are released, so the hand-off flag to the IEKF stream goes up now, with
  // the margi head's number (no k_sync_set launch between the two kernels)
  if (tail_flag && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(tail_flag, (unsigned)st->margi_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int lane = threadIdx.x & 63;
  const int nl = *nleaves;
  if (exist_up)
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nl; q += gridDim.x * blockDim.x) {
      const int node = leaves[q];
      margi_exist_up(m, node, m.hdr[node].isexist ? 1 : 0);
    }
  const int s0 = win->mp[0];
  const M3 R0 = ld_m3(win->R[0]);
  const V3 p0 = ld_v3(win->p[0]);
  for (int q = blockIdx.x * kCopyWaves + (threadIdx.x >> 6); q < nl; q += gridDim.x * kCopyWaves) {
    const int* pq = &plan[(size_t)q * 8];
    const int src = pq[0], segn = pq[4];
    if (src >= 0) {
      const int nold = pq[1], dst = pq[2];
      for (int j = lane; j < nold; j += 64) {
        const size_t a = (size_t)src + j, b = (size_t)dst + j;
        for (int t = 0; t < 3; t++) m.fix_pnt[b * 3 + t] = m.fix_pnt[a * 3 + t];
        for (int t = 0; t < 9; t++) m.fix_var[b * 9 + t] = m.fix_var[a * 9 + t];
      }
    }
    if (segn > 0) {
      const int seg = pq[3], dst = pq[5];
      for (int j = lane; j < segn; j += 64) {
        const int i = m.wp_ord[(size_t)s0 * m.ord_stride + seg + j];
        const size_t b = (size_t)s0 * m.cap_wp + i;
        const V3 pt = rigid(R0, ld_v3(&m.wp_pnt[b * 3]), p0);
        const size_t d = (size_t)dst + j;
        for (int t = 0; t < 3; t++) m.fix_pnt[d * 3 + t] = pt[t];
        for (int t = 0; t < 9; t++) m.fix_var[d * 9 + t] = m.wp_var[b * 9 + t];
      }
    }
  }
}

// internal nodes bottom-up: isexist = OR(children) (octree.cpp:485-494); the
// deepest level's launch also clears the oldest-slot segment records
__device__ __forceinline__ void internal_exist(DevMap& m, int node) {
  NodeHdr& h = m.hdr[node];
  if (h.octo != 1) return;
  int8_t e = 0;
  for (int o = 0; o < 8; o++)
    if (h.child[o] >= 0) e |= m.hdr[h.child[o]].isexist;
  h.isexist = e ? 1 : 0;
}
__global__ void __launch_bounds__(256) k_margi_internal(int L, int thread_num, DevMap m, int* __restrict__ lists,
                                                        const int* __restrict__ rc, const int* __restrict__ gate) {
  if (gate && !*gate) return;  // a speculative tail the LM did not reach (ba_run)
  if (g_slide(m) < thread_num) return;
  int* work;
  const int nw = margi_level(L, m, rc, lists, &work);
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nw; q += gridDim.x * blockDim.x) internal_exist(m, work[q]);
}

// erase dead roots from surf_map_slide (local_mapping.cpp:67-78) with
// clear_slwd over their subtrees (octree.cpp:739-756), top-down. Level 0 also
// finishes the bottom-up isexist pass (its roots are level 0's own nodes);
// level L also resets the dead marks of level L-2, which nobody reads any more.
__global__ void __launch_bounds__(256) k_margi_erase_mark(int L, int thread_num, DevMap m, int* __restrict__ lists,
                                                          const int* __restrict__ rc, const int* __restrict__ gate) {
  if (gate && !*gate) return;  // a speculative tail the LM did not reach (ba_run)
  if (g_slide(m) < thread_num) return;
  int* work;
  const int nw = margi_level(L, m, rc, lists, &work);
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nw; q += gridDim.x * blockDim.x) {
    int node = work[q];
    NodeHdr& h = m.hdr[node];
    int dead;
    if (L == 0) {
      internal_exist(m, node);
      dead = h.isexist ? 0 : 1;
    } else {
      dead = m.nscr[(size_t)h.parent * 4 + 2] == 7 ? 1 : 0;
    }
    if (dead) {
      m.nscr[(size_t)node * 4 + 2] = 7;
      h.has_sw = 0;
      for (int j = 0; j < m.W; j++) clu_zero(m.pcrs[(size_t)node * m.W + j]);
      if (L == 0) m.in_slide[node] = 0;
    }
  }
  if (L >= 2) {
    const int nc = margi_level(L - 2, m, rc, lists, &work);
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nc; q += gridDim.x * blockDim.x)
      m.nscr[(size_t)work[q] * 4 + 2] = -1;
  }
}
// reset the dead marks of levels L0 .. nlev-1
__global__ void __launch_bounds__(256) k_clear_mark(int L0, int nlev, int thread_num, DevMap m,
                                                    int* __restrict__ lists, const int* __restrict__ rc, const int* __restrict__ gate) {
  if (gate && !*gate) return;  // a speculative tail the LM did not reach (ba_run)
  if (g_slide(m) < thread_num) return;
  for (int L = L0 < 0 ? 0 : L0; L < nlev; L++) {
    int* work;
    const int nw = margi_level(L, m, rc, lists, &work);
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nw; q += gridDim.x * blockDim.x)
      m.nscr[(size_t)work[q] * 4 + 2] = -1;
  }
}
// local_mapping.cpp:67-78 + clear_slwd (octree.cpp:739-756) in one launch: a
// node of the slide subtrees is erased with its root, so every node of every
// level looks its root up (L parent hops) — the roots' isexist is final
// (margi_exist_up) — instead of a top-down launch per level with dead marks
__global__ void __launch_bounds__(256) k_margi_erase_all(int nlev, int thread_num, DevMap m, const int* __restrict__ lists,
                                                         const int* __restrict__ rc, const int* __restrict__ gate) {
  if (gate && !*gate) return;  // a speculative tail the LM did not reach (ba_run)
  if (g_slide(m) < thread_num) return;
  const int n0 = m.counters[kCntSlide];
  int total = n0;
  for (int l = 1; l < nlev; l++) total += rc[l - 1];
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < total; q += gridDim.x * blockDim.x) {
    int L = 0, node;
    if (q < n0) {
      node = m.slide[q];
    } else {
      int r = q - n0, off = 0;
      L = 1;
      while (L < nlev - 1 && r >= rc[L - 1]) {
        r -= rc[L - 1];
        off += rc[L - 1];
        L++;
      }
      node = lists[off + r];
    }
    int root = node;
    for (int k = 0; k < L; k++) root = m.hdr[root].parent;
    if (!m.hdr[root].isexist) {
      m.hdr[node].has_sw = 0;
      for (int j = 0; j < m.W; j++) clu_zero(m.pcrs[(size_t)node * m.W + j]);
      if (L == 0) m.in_slide[node] = 0;
    }
  }
}

// single block, order-preserving in-place compaction of the slide list (a
// chunk is read completely before any of it is written; writes never pass
// the read position)
// then (the same workgroup) the x_buf / imu_pre_buf slide of the device state
// (local_mapping.cpp:536-546) and the end-of-scan counter publication
__global__ void __launch_bounds__(1024) k_slide_compact(int thread_num, DevMap m, DState* __restrict__ st, int wc,
                                                        int nimu, Pub* __restrict__ pub, int seq2, const int* __restrict__ gate) {
  if (gate && !*gate) return;  // a speculative tail the LM did not reach (ba_run)
  if (threadIdx.x == 0 && st->jour_check && wc > 0) {  // local_mapping.cpp:510-518, x_curr.p = x_buf.back().p
    const double* xb = st->xs + (size_t)(wc - 1) * kXS + 9;  // (read before the slide below)
    const V3 p = v3(xb[0], xb[1], xb[2]);
    const double spat = norm3(sub(p, v3(st->last_pos[0], st->last_pos[1], st->last_pos[2])));
    if (spat > 0.5) {
      st->jour += spat;
      for (int j = 0; j < 3; j++) st->last_pos[j] = p[j];
    }
    st->jour_check = 0;
  }
  __shared__ int base;
  __shared__ int sc[1024];
  __shared__ int s_w[17];
  const int n = m.counters[kCntSlide];
  constexpr int kPer = 16;
  if (g_slide(m) >= thread_num && n <= kPer * (int)blockDim.x) {
    // one pass: every lane reads a contiguous run into registers, one block
    // scan orders the survivors (all reads precede the scan's barriers, so the
    // in-place writes cannot overtake them)
    const int per = (n + (int)blockDim.x - 1) / (int)blockDim.x;
    const int q0 = threadIdx.x * per;
    int nodes[kPer];
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const int q = q0 + k;
      int node = (k < per && q < n) ? m.slide[q] : -1;
      if (node >= 0 && !m.in_slide[node]) node = -1;
      nodes[k] = node;
      cnt += node >= 0 ? 1 : 0;
    }
    int total;
    int pos = block_excl_scan(cnt, s_w, &total);
#pragma unroll
    for (int k = 0; k < kPer; k++)
      if (nodes[k] >= 0) m.slide[pos++] = nodes[k];
    if (threadIdx.x == 0) m.counters[kCntSlide] = total;
  } else if (g_slide(m) >= thread_num) {
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    for (int start = 0; start < n; start += blockDim.x) {
      const int q = start + threadIdx.x;
      const int node = q < n ? m.slide[q] : -1;
      const int keep = (node >= 0 && m.in_slide[node]) ? 1 : 0;
      sc[threadIdx.x] = keep;
      __syncthreads();
      for (int off = 1; off < (int)blockDim.x; off <<= 1) {
        int v = threadIdx.x >= (unsigned)off ? sc[threadIdx.x - off] : 0;
        __syncthreads();
        sc[threadIdx.x] += v;
        __syncthreads();
      }
      if (keep) m.slide[base + sc[threadIdx.x] - 1] = node;
      __syncthreads();
      if (threadIdx.x == blockDim.x - 1) base += sc[threadIdx.x];
      __syncthreads();
    }
    if (threadIdx.x == 0) m.counters[kCntSlide] = base;
  }
  const int t = threadIdx.x;
  const double v = (t < (wc - 1) * kXS) ? st->xs[kXS + t] : 0.0;
  const double b = (t < (nimu - 1) * 12) ? st->bias[12 + t] : 0.0;
  __syncthreads();
  if (t < (wc - 1) * kXS) st->xs[t] = v;
  if (t < (nimu - 1) * 12) st->bias[t] = b;
  if (t == 0) st->imu_head = (st->imu_head + 1) % kMaxWin;  // imu_pre_buf.pop_front (the record ring)
  if (seq2 < 0) seq2 = st->seq2;  // set by k_make_win (replayed graph)
  if (seq2 > 0) {
    __syncthreads();
    if (t < kCntN) pub_store(&pub->counters[t], m.counters[t]);
    pub_drain();
    __syncthreads();
    if (t == 0) pub_flag(&pub->seq2, seq2);
  }
}
__global__ void __launch_bounds__(256) k_set_jour(int thread_num, DevMap m, const double* __restrict__ jour,
                                                  int* __restrict__ rc, int n_oldest) {
  if (blockIdx.x == 0) {  // margi level counts and the leaf count start at zero
    // kRcStatus is the recut's (k_ba_init may read it concurrently on the main stream)
    for (int i = threadIdx.x; i < kRcN; i += blockDim.x)
      if (i != kRcStatus) rc[i] = (i == kRcNOld) ? n_oldest : 0;
    if (threadIdx.x == 0) m.counters[kCntLeaves] = 0;
  }
  const int n = m.counters[kCntSlide];
  if (g_slide(m) < thread_num) return;
  const double j = *jour;  // the device's jour (DState::jour, the previous margi's update)
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) m.jour[m.slide[q]] = j;
}

// multi_margi (local_mapping.cpp:21-78): every count stays on the device;
// the host enqueues max_layer+1 levels (no level can be deeper) and
// synchronises once at the end for the error flags.
// The part of multi_margi that does not depend on the BA (jour stamps, the
// slide-tree levels, the oldest slot's points grouped by leaf), enqueued right
// after the recut on the second stream so it runs under the LM iterations.
int map_margi_prefix(vg_ctx* ctx, const MP& mp, int slot0, int n_oldest, int thread_num, const unsigned* flags) {
  DevMap& m = ctx->map;
  Work& w = ctx->wk;
  hipStream_t s = ctx->stream_ds;
  const int nlev = mp.max_layer + 1;
  if (flags) {  // the scan graph: k_ba_init raises d_sync[3] once the recut has ended (no event inside a graph)
    VG_TRY(sync_wait(ctx, s, 3, flags[0]));
  } else {
    VG_HIP(flush_insert_events(ctx));
    VG_HIP(hipStreamWaitEvent(s, ctx->ev_recut_done, 0));  // recorded at the recut's end (map_recut)
  }
  const int gl = 64;  // grid-stride over device-side counts
  k_set_jour<<<gl, kBlock, 0, s>>>(thread_num, m, &ctx->st->jour, w.rc, n_oldest);
  for (int L = 0; L < nlev; L++) k_collect_level<<<gl * (kBlock / kSpreadBlock), kSpreadBlock, 0, s>>>(L, thread_num, m, w.list1, w.list0, w.rc);
  (void)slot0;  // the oldest slot's points per leaf are the leaves' runs (DevMap::lseg): no sort here
  (void)n_oldest;
  VG_HIP(hipGetLastError());
  if (flags) VG_TRY(sync_set(ctx, s, 4, flags[1]));  // the scan graph's margi tail waits for it
  VG_HIP(hipEventRecord(ctx->ev_prefix_done, s));
  return VG_OK;
}

// pub_localmap's /map_cmap cloud (publishers.cpp:102-119): every third point
// of the oldest window frame (mgsize = 1: pvec_buf[0]) at x_buf[0] after the
// BA, R pnt + p in fp64, stored as float like the PointType it publishes
__global__ void __launch_bounds__(256) k_local_map(const WinD* __restrict__ win, DevMap m, float4* __restrict__ out,
                                                   int* __restrict__ nout, const int* __restrict__ gate) {
  if (gate && !*gate) return;  // a speculative tail the LM did not reach (ba_run)
  const int slot = win->mp[0];
  const int n = m.wpn[slot];
  const int nk = (n + 2) / 3;
  if (blockIdx.x == 0 && threadIdx.x == 0) nout[0] = nk;
  const M3 R = ld_m3(win->R[0]);
  const V3 p = ld_v3(win->p[0]);
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < nk; k += gridDim.x * blockDim.x) {
    const size_t b = (size_t)slot * m.cap_wp + 3 * k;
    const V3 w = rigid(R, ld_v3(&m.wp_pnt[b * 3]), p);
    out[k] = make_float4((float)w[0], (float)w[1], (float)w[2], m.wp_int[b]);
  }
}

int map_margi(vg_ctx* ctx, const MP& mp, const WinArg& wa, int n_oldest, int thread_num, int pub_seq,
              int pub_seq2, const int* gate) {
  DevMap& m = ctx->map;
  Work& w = ctx->wk;
  hipStream_t s = ctx->stream;
  const int nlev = mp.max_layer + 1;
  WinD* dwin = (WinD*)ctx->ba.xs;
  int* dn = (int*)((char*)ctx->ba.xs + sizeof(WinD));
  if (wa.win_count * kXS > 1024) {
    ctx->err = "win_size too large for the state slide";
    return VG_E_ARG;
  }
  // x_curr.R/p <- x_buf.back() and the window view (which also stores the
  // end-of-scan publication number); the state is then final for this scan
  // and is published — all by k_margi_leaf's workgroup 0, beside the leaves
  WinArg wa2 = wa;
  wa2.seq2 = pub_seq2;
  VG_HIP(hipStreamWaitEvent(s, ctx->ev_prefix_done, 0));  // map_margi_prefix
  // the rest reads every per-scan value from the device (n_oldest: rc, the
  // publication number: the state), so it is captured once and replayed
  const int gl = 64;
  // k_margi_leaf's plane updates are the last margi work the next scan's
  // IEKF reads: ev_tail_a marks them, and the remainder (point_fix copies,
  // isexist / erase marks, slide compaction, the device-state slide, the
  // counter publication; nothing the IEKF reads) runs under the next IEKF
  // one lane per leaf (eigen-decomposition + plane_update in series on the lane):
  // enough blocks that no lane takes two leaves, surplus blocks exit at once
  // workgroup 0 is the margi head (the window view and the state publication,
  // k_make_win_publish's work) running beside the leaves
  const int* bi = pub_seq > 0 ? ba_iters_dev(ctx) : nullptr;
  // the hand-off flags to the next scan's IEKF stream: the margi head's
  // x_curr (d_sync[2], the device propagation starts from it) and the leaves'
  // plane updates (d_sync[0], the IEKF reads them)
  // (sharded as well: the hand-offs are device-side only, and no exchange sits
  // between a flag's producer and its consumer)
  const bool flags = ctx->flag_sync && ctx->overlap_iekf && ctx->use_graphs && !ctx->prof_stages;
  k_margi_leaf<<<1 + 512 * kBlock / kSpreadBlock, kSpreadBlock, 0, s>>>(
      m.counters + kCntLeaves, w.list0, mp, wa2, ctx->st, dwin, dn, dn + 32, bi != nullptr, bi,
      bi ? ba_hess_dev(ctx) : nullptr, ctx->d_pub, pub_seq, m, ctx->ba.fac_eig, ctx->ba.fac_pcr, w.plan, gate,
      flags ? ctx->d_sync + 2 : nullptr, ctx->margi_batch ? 1 : 0, nullptr, nullptr);
  VG_HIP(hipEventRecord(ctx->ev_tail_a, s));
  // the margi's publication number into the IEKF hand-off flag: by the margi
  // graph's first kernel (k_margi_copy) — or k_sync_set when the local map
  // publication sits in between
  const bool copy_signals = flags && !(ctx->pub_flags & 1);
  if (flags && !copy_signals) VG_TRY(sync_set(ctx, s, 0, (unsigned)pub_seq, gate));
  if (ctx->pub_flags & 1) k_local_map<<<64, kBlock, 0, s>>>(dwin, m, ctx->d_cmap, ctx->d_cmap_n, gate);
  ctx->tail_a_valid = true;
  auto body = [&]() -> int {
    const bool fused = ctx->margi_fused;
    k_margi_copy<<<256, 64 * kCopyWaves, 0, s>>>(m.counters + kCntLeaves, w.plan, dwin, m, gate, w.list0, fused ? 1 : 0,
                                                  copy_signals ? ctx->d_sync : nullptr, ctx->st);
    if (fused) {
      k_margi_erase_all<<<gl * (kBlock / kSpreadBlock), kSpreadBlock, 0, s>>>(nlev, thread_num, m, w.list1, w.rc, gate);
    } else {
      for (int L = nlev - 1; L >= 1; L--)
        k_margi_internal<<<gl * (kBlock / kSpreadBlock), kSpreadBlock, 0, s>>>(L, thread_num, m, w.list1, w.rc, gate);
      for (int L = 0; L < nlev; L++)
        k_margi_erase_mark<<<gl * (kBlock / kSpreadBlock), kSpreadBlock, 0, s>>>(L, thread_num, m, w.list1, w.rc, gate);
      k_clear_mark<<<gl, kBlock, 0, s>>>(nlev - 2, nlev, thread_num, m, w.list1, w.rc, gate);
    }
    // slide list compaction, the device-state slide, the counter publication
    k_slide_compact<<<1, 1024, 0, s>>>(thread_num, m, ctx->st, wa.win_count, mp.W - 1, ctx->d_pub, -1, gate);
    VG_HIP(hipGetLastError());
    return VG_OK;
  };
  (void)n_oldest;
  if (!ctx->use_graphs || ctx->prof_stages) return body();
  hipGraphExec_t& ge = ctx->g_margi[(gate ? 1 : 0) + (copy_signals ? 2 : 0)];
  if (!ge) {
    std::lock_guard<std::recursive_mutex> cap_lk_(capture_mutex());  // (vg_internal.h)
    VG_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    const int r = body();
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(s, &g);
    if (r != VG_OK) return r;
    VG_HIP(e);
    VG_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    VG_HIP(hipGraphDestroy(g));
  }
  VG_HIP(hipGraphLaunch(ge, s));
  return VG_OK;  // device error flags reach the host with the end-of-scan counters
}

// The margi tail inside the scan graph (pipeline.cpp stage_insert_recut),
// captured on the context stream behind the first two LM iterations: gated on
// the LM's `fin` like a speculative tail; the margi prefix (second stream) is
// waited for on a device flag (d_sync[4] >= DState::ph[4], by k_margi_leaf's
// leaf workgroups: no polling kernel in front); the publication
// numbers come from DState::ph; the ring (wa) is the graph's own.
int map_margi_tail_capture(vg_ctx* ctx, const MP& mp, const WinArg& wa) {
  DevMap& m = ctx->map;
  Work& w = ctx->wk;
  hipStream_t s = ctx->stream;
  const int nlev = mp.max_layer + 1;
  WinD* dwin = (WinD*)ctx->ba.xs;
  int* dn = (int*)((char*)ctx->ba.xs + sizeof(WinD));
  const int* gate = ba_gate_dev(ctx);
  const int thread_num = ctx->cfg.thread_num;
  k_margi_leaf<<<1 + 512 * kBlock / kSpreadBlock, kSpreadBlock, 0, s>>>(
      m.counters + kCntLeaves, w.list0, mp, wa, ctx->st, dwin, dn, dn + 32, 1, ba_iters_dev(ctx), ba_hess_dev(ctx),
      ctx->d_pub, 0, m, ctx->ba.fac_eig, ctx->ba.fac_pcr, w.plan, gate, ctx->d_sync + 2, ctx->margi_batch ? 1 : 0,
      &ctx->st->ph[1], ctx->d_sync + 4);
  k_margi_copy<<<256, 64 * kCopyWaves, 0, s>>>(m.counters + kCntLeaves, w.plan, dwin, m, gate, w.list0,
                                                ctx->margi_fused ? 1 : 0, ctx->d_sync, ctx->st);
  if (ctx->margi_fused) {
    k_margi_erase_all<<<64 * (kBlock / kSpreadBlock), kSpreadBlock, 0, s>>>(nlev, thread_num, m, w.list1, w.rc, gate);
  } else {
    for (int L = nlev - 1; L >= 1; L--)
      k_margi_internal<<<64 * (kBlock / kSpreadBlock), kSpreadBlock, 0, s>>>(L, thread_num, m, w.list1, w.rc, gate);
    for (int L = 0; L < nlev; L++)
      k_margi_erase_mark<<<64 * (kBlock / kSpreadBlock), kSpreadBlock, 0, s>>>(L, thread_num, m, w.list1, w.rc, gate);
    k_clear_mark<<<64, kBlock, 0, s>>>(nlev - 2, nlev, thread_num, m, w.list1, w.rc, gate);
  }
  k_slide_compact<<<1, 1024, 0, s>>>(thread_num, m, ctx->st, wa.win_count, mp.W - 1, ctx->d_pub, -1, gate);
  VG_HIP(hipGetLastError());
  return VG_OK;
}

}  // namespace vg

#ifdef VG_PROBE
VG_PROBE_READER(vg_probe_read_map)
#endif
