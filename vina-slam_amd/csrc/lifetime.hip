// lifetime.hip — the map's lifetime: the journey release and the reclaim of
// erased nodes and abandoned point_fix blocks.
//
// The reference erases, in its idle branch, every root voxel whose jour stamp
// is >= 700 m behind (local_mapping.cpp:317-344, OctoTree::tras_ptr,
// octree.cpp:597-608) and frees a leaf's point_fix once it reaches max_points
// (octree.cpp:467-468); its heap takes the memory back. The device map is a
// node pool with a bump counter and a point_fix arena with bump-allocated
// blocks (a growing leaf abandons its old block, map.hip k_margi_leaf), so the
// release here is: mark the erased roots (a root hash pass), mark every node by
// its root (parent hops), then compact the pool and the arena in place,
// order-preserving (an exclusive scan of the live flags is the new id of every
// node: relative id order — k_fac_sort's factor order — is unchanged), remap
// every node reference that outlives a scan (children, parents, the root hash,
// the slide list, the window points' leaves) and rebuild the hash. Every array
// is gathered into a scratch buffer and copied back; the freed tail is put back
// in the state map_reset leaves it in (records handed out zeroed).
// Runs between scans only (vg_release_far completes the outstanding work first).
#include <hipcub/hipcub.hpp>
#include "vg_dev.h"

namespace vg {

namespace {
enum { kRelDead = 0, kRelRootsLive = 1, kRelNodesDead = 2, kRelGarbage = 3, kRelFixHeld = 4, kRelKeys = 5, kRelN = 8 };

// roots: 1 erased, 2 kept (hashed or in the slide list); 0: not a root / not hashed
__global__ void __launch_bounds__(256) k_rel_mark(DevMap m, int n, int nslide, int release, int thr, double jour,
                                                  int* __restrict__ mark, unsigned long long* __restrict__ cnt) {
  const int hs = m.hash_mask + 1;
  const int stride = gridDim.x * blockDim.x;
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < hs; s += stride) {
    if (m.hkey[s] == kKeyEmpty) continue;
    const int r = m.hval[s];
    if (r < 0 || r >= n) continue;
    // local_mapping.cpp:323-324: int dis = jour - iter->second->jour; dis < 700 keeps
    const int dis = (int)(jour - m.jour[r]);
    const bool dead = release && !m.in_slide[r] && dis >= thr;
    mark[r] = dead ? 1 : 2;
    atomicAdd(&cnt[dead ? kRelDead : kRelRootsLive], 1ull);
  }
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nslide; q += stride) {
    const int r = m.slide[q];
    if (r >= 0 && r < n) mark[r] = 2;  // (a slide root is never erased: it is hashed and marked 2 above)
  }
}

// per node: live (its root kept), its point_fix block to keep (fix_cap while
// fix_cnt > 0; a leaf past max_points keeps no block, octree.cpp:467-468)
__global__ void __launch_bounds__(256) k_rel_live(DevMap m, int n, const int* __restrict__ mark, int* __restrict__ live,
                                                  int* __restrict__ fblk, unsigned long long* __restrict__ cnt) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int r = i;
    for (int k = 0; k < 8; k++) {  // depth <= max_layer + 1 <= 4 (vg_create rejects max_layer > 3)
      const int p = m.hdr[r].parent;
      if (p < 0) break;
      r = p;
    }
    const int mk = m.hdr[r].parent < 0 ? mark[r] : 0;
    const int l = mk == 2 ? 1 : 0;
    live[i] = l;
    const NodeHdr& h = m.hdr[i];
    fblk[i] = (l && h.fix_cnt > 0) ? h.fix_cap : 0;
    if (mk == 1) atomicAdd(&cnt[kRelNodesDead], 1ull);
    if (mk == 0) atomicAdd(&cnt[kRelGarbage], 1ull);
    if (l && h.fix_cnt > 0) atomicAdd(&cnt[kRelFixHeld], (unsigned long long)h.fix_cnt);
  }
}

// The root hash rebuilt from the kept roots with a layout that is a function
// of the kept (key, new id) set alone, not of scheduling: each kept root's key
// is filed under its new id (ids are unique, no atomics), the table is
// cleared, then linear probing runs in rounds — every unplaced root bids for
// its current probe slot with atomicMin of its id (in hfirst, which must end
// cleared anyway), the lowest id takes the slot, the others move one slot on.
// A winner never moves again, so every slot between a root's home and its
// final slot is occupied: hash_find's probe sequence stays valid.
__global__ void __launch_bounds__(256) k_rel_hash_collect(DevMap m, int n, const int* __restrict__ live,
                                                          const int* __restrict__ nid, uint64_t* __restrict__ rkey,
                                                          int* __restrict__ pos) {
  const int hs = m.hash_mask + 1;
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < hs; s += gridDim.x * blockDim.x) {
    const uint64_t key = m.hkey[s];
    if (key == kKeyEmpty) continue;
    const int r = m.hval[s];
    if (r < 0 || r >= n || !live[r]) continue;
    const int q = nid[r];
    rkey[q] = key;
    pos[q] = (int)hash_slot(key, m.hash_mask);  // its home slot; -1 (memset) for every other id
  }
}
// one probing round: bids (phase 0), then the outcome (phase 1); cnt: roots
// still unplaced after the round (each counted once: moved on in phase 0 or
// outbid in phase 1)
constexpr int kBid = 1 << 30;  // pos[q] flag: q bid for that slot in this round's phase 0
__global__ void __launch_bounds__(256) k_rel_hash_round(DevMap m, int nl, const uint64_t* __restrict__ rkey,
                                                        int* __restrict__ pos, int phase, int* __restrict__ cnt) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nl; q += gridDim.x * blockDim.x) {
    int p = pos[q];
    if (p < 0) continue;  // not a kept root, or placed
    if (phase == 0) {
      if (m.hkey[p] != kKeyEmpty) {  // a winner of an earlier round: probe on (bid next round)
        pos[q] = (p + 1) & m.hash_mask;
        atomicAdd(cnt, 1);
      } else {
        atomicMin(&m.hfirst[p], q);
        pos[q] = p | kBid;
      }
      continue;
    }
    if (!(p & kBid)) continue;
    p &= ~kBid;
    if (m.hfirst[p] == q) {  // won: the lowest id bidding for the slot
      m.hkey[p] = rkey[q];
      m.hval[p] = q;
      pos[q] = -1;
      m.hfirst[p] = 0x7f7f7f7f;  // an outbid lane reading it after this still sees != its id
    } else {
      pos[q] = (p + 1) & m.hash_mask;
      atomicAdd(cnt, 1);
    }
  }
}

// one per-node array of `w` 32-bit words per node: the live records to their new ids
__global__ void __launch_bounds__(256) k_rel_gather(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int w,
                                                    long total, const int* __restrict__ live, const int* __restrict__ nid) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int i = (int)(e / w);
    if (live[i]) dst[(size_t)nid[i] * w + (e - (long)i * w)] = src[e];
  }
}
__global__ void __launch_bounds__(256) k_rel_gather_u8(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int n,
                                                       const int* __restrict__ live, const int* __restrict__ nid) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    if (live[i]) dst[nid[i]] = src[i];
}
// the node records with their references remapped: children, parent, the point_fix block
__global__ void __launch_bounds__(256) k_rel_hdr(DevMap m, int n, const int* __restrict__ live, const int* __restrict__ nid,
                                                 const int* __restrict__ fblk, const int* __restrict__ foff,
                                                 NodeHdr* __restrict__ out) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (!live[i]) continue;
    NodeHdr h = m.hdr[i];
    for (int k = 0; k < 8; k++) h.child[k] = h.child[k] >= 0 ? nid[h.child[k]] : -1;
    h.parent = h.parent >= 0 ? nid[h.parent] : -1;
    if (fblk[i] > 0) {
      h.fix_off = foff[i];
      h.fix_cap = fblk[i];
    } else {
      h.fix_off = 0;
      h.fix_cap = 0;
      h.fix_cnt = 0;
    }
    out[nid[i]] = h;
  }
}
// a kept point_fix block (its fix_cnt points, `w` doubles each) to its new offset; one wave per node
__global__ void __launch_bounds__(256) k_rel_fix(DevMap m, int n, const double* __restrict__ src, int w,
                                                 const int* __restrict__ fblk, const int* __restrict__ foff,
                                                 double* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const int wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
  for (int i = wid; i < n; i += nw) {
    if (fblk[i] <= 0) continue;
    const NodeHdr& h = m.hdr[i];
    const size_t a = (size_t)h.fix_off * w, b = (size_t)foff[i] * w, cnt = (size_t)h.fix_cnt * w;
    for (size_t e = lane; e < cnt; e += 64) dst[b + e] = src[a + e];
  }
}
// node ids held outside the pool: the slide list (all kept) and the window points' leaves
__global__ void __launch_bounds__(256) k_rel_remap(int* __restrict__ ids, long n, int nnodes, const int* __restrict__ live,
                                                   const int* __restrict__ nid) {
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x) {
    const int v = ids[q];
    if (v >= 0 && v < nnodes) ids[q] = live[v] ? nid[v] : -1;
  }
}
__global__ void k_rel_counts(DevMap m, int n_live, int fix_used) {
  if (threadIdx.x == 0) {
    m.counters[kCntNodes] = n_live;
    m.counters[kCntFix] = fix_used;
  }
}

// test hook (vgx_roots): per node, its subtree's root gets the node and its point_fix points
__global__ void __launch_bounds__(256) k_roots_count(DevMap m, int n, int* __restrict__ nodes, int* __restrict__ nfix) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int r = i;
    for (int k = 0; k < 16 && m.hdr[r].parent >= 0; k++) r = m.hdr[r].parent;
    if (m.hdr[r].parent >= 0) continue;
    atomicAdd(&nodes[r], 1);
    const int f = m.hdr[i].fix_cnt;
    if (f > 0) atomicAdd(&nfix[r], f);
  }
}
// one row per hashed root: key x/y/z, jour stamp, flags (1 in the slide map, 2 isexist), subtree counts
__global__ void __launch_bounds__(256) k_roots_rows(DevMap m, int n, const int* __restrict__ nodes,
                                                    const int* __restrict__ nfix, int* __restrict__ cnt,
                                                    long long* __restrict__ key, double* __restrict__ jour,
                                                    int* __restrict__ flags, int* __restrict__ onodes,
                                                    int* __restrict__ ofix) {
  const int hs = m.hash_mask + 1;
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < hs; s += gridDim.x * blockDim.x) {
    const uint64_t k = m.hkey[s];
    if (k == kKeyEmpty) continue;
    const int r = m.hval[s];
    if (r < 0 || r >= n) continue;
    const int q = atomicAdd(cnt, 1);
    key[3 * q] = unpack_axis(k, 42);
    key[3 * q + 1] = unpack_axis(k, 21);
    key[3 * q + 2] = unpack_axis(k, 0);
    jour[q] = m.jour[r];
    flags[q] = (m.in_slide[r] ? 1 : 0) | (m.hdr[r].isexist ? 2 : 0);
    onodes[q] = nodes[r];
    ofix[q] = nfix[r];
  }
}

template <class F>
int with_scratch(vg_ctx* ctx, size_t bytes, void** p, F&& body) {
  const hipError_t e = hipMalloc(p, bytes > 0 ? bytes : 64);
  if (e != hipSuccess) {
    ctx->err = std::string("vg_release_far: scratch (") + std::to_string(bytes >> 20) + " MiB): " + hipGetErrorString(e);
    return VG_E_HIP;
  }
  const int r = body();
  const hipError_t e2 = hipStreamSynchronize(ctx->stream);
  (void)hipFree(*p);
  if (r != VG_OK) return r;
  if (e2 != hipSuccess) {
    ctx->err = std::string("vg_release_far: ") + hipGetErrorString(e2);
    return VG_E_HIP;
  }
  return VG_OK;
}
}  // namespace

int map_release(vg_ctx* ctx, bool release, int thr, double jour, int compact, long long* out) {
  DevMap& m = ctx->map;
  hipStream_t s = ctx->stream;
  // every stream of the context is idle before the map is rewritten in place
  // (host_sync drains the main stream, which waits for the others' work of
  // the pipeline; the downsample and IEKF streams are drained here as well)
  VG_HIP(hipStreamSynchronize(ctx->stream_ds));
  if (ctx->stream_iekf) VG_HIP(hipStreamSynchronize(ctx->stream_iekf));
  int hc[kCntN];
  VG_HIP(hipMemcpyAsync(hc, m.counters, sizeof(hc), hipMemcpyDeviceToHost, s));
  VG_HIP(hipStreamSynchronize(s));
  const int n = hc[kCntNodes] < m.cap_nodes ? hc[kCntNodes] : m.cap_nodes;
  const int nslide = hc[kCntSlide], nfix_used = hc[kCntFix];
  const size_t un = (size_t)(n > 0 ? n : 1);
  size_t tb = 0;
  VG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (int*)nullptr, (int*)nullptr, (int)un, s));
  // scratch: counters, then per node mark / live / new id / kept block / new offset, the scan workspace
  const size_t off_cnt = 0, off_mark = 256, off_live = off_mark + un * 4, off_nid = off_live + un * 4,
               off_fblk = off_nid + un * 4, off_foff = off_fblk + un * 4, off_tmp = ((off_foff + un * 4 + 255) / 256) * 256;
  void* sp = nullptr;
  unsigned long long hcnt[kRelN] = {0};
  int n_live = 0, fix_new = 0;
  bool did = false;
  const int r = with_scratch(ctx, off_tmp + tb, &sp, [&]() -> int {
    char* b = (char*)sp;
    auto* cnt = (unsigned long long*)(b + off_cnt);
    int *mark = (int*)(b + off_mark), *live = (int*)(b + off_live), *nid = (int*)(b + off_nid);
    int *fblk = (int*)(b + off_fblk), *foff = (int*)(b + off_foff);
    VG_HIP(hipMemsetAsync(b, 0, off_live, s));  // counters + marks
    const int g = grid_for(std::max((long)m.hash_mask + 1, (long)n));
    k_rel_mark<<<g, kBlock, 0, s>>>(m, n, nslide, release ? 1 : 0, thr, jour, mark, cnt);
    if (n > 0) {
      k_rel_live<<<grid_for(n), kBlock, 0, s>>>(m, n, mark, live, fblk, cnt);
      size_t t2 = tb;
      VG_HIP(hipcub::DeviceScan::ExclusiveSum(b + off_tmp, t2, live, nid, n, s));
      VG_HIP(hipcub::DeviceScan::ExclusiveSum(b + off_tmp, t2, fblk, foff, n, s));
    }
    VG_HIP(hipGetLastError());
    int tail[4] = {0, 0, 0, 0};
    VG_HIP(hipMemcpyAsync(hcnt, cnt, sizeof(hcnt), hipMemcpyDeviceToHost, s));
    if (n > 0) {
      VG_HIP(hipMemcpyAsync(&tail[0], nid + n - 1, sizeof(int), hipMemcpyDeviceToHost, s));
      VG_HIP(hipMemcpyAsync(&tail[1], live + n - 1, sizeof(int), hipMemcpyDeviceToHost, s));
      VG_HIP(hipMemcpyAsync(&tail[2], foff + n - 1, sizeof(int), hipMemcpyDeviceToHost, s));
      VG_HIP(hipMemcpyAsync(&tail[3], fblk + n - 1, sizeof(int), hipMemcpyDeviceToHost, s));
    }
    VG_HIP(hipStreamSynchronize(s));
    n_live = tail[0] + tail[1];
    fix_new = tail[2] + tail[3];
    // compact when the release erased something, when asked, or when over half
    // of the point_fix arena is abandoned blocks
    const bool go = n > 0 && (hcnt[kRelDead] > 0 || hcnt[kRelGarbage] > 0 || compact ||
                              (long)nfix_used > 2l * (long)fix_new);
    if (!go) return VG_OK;
    did = true;
    // the gather buffer: the largest per-node array of the kept nodes, the kept point_fix blocks, the hash pairs
    const int W = m.W;
    const size_t rec_max = std::max({sizeof(NodeHdr), sizeof(PlaneRec), (size_t)kCovN * 8, (size_t)W * sizeof(Clu),
                                     (size_t)W * sizeof(uint64_t)});
    const size_t gbytes = std::max({(size_t)n_live * rec_max, (size_t)fix_new * 9 * sizeof(double),
                                    (size_t)n_live * 12 + 64});
    void* gp = nullptr;
    return with_scratch(ctx, gbytes, &gp, [&]() -> int {
      // the root hash, rebuilt from the kept roots under their new ids, its
      // layout a function of the kept set (k_rel_hash_collect)
      auto* rkey = (uint64_t*)gp;
      int* pos = (int*)(rkey + n_live);
      const int gh = grid_for((long)m.hash_mask + 1);
      VG_HIP(hipMemsetAsync(pos, 0xff, (size_t)n_live * sizeof(int), s));
      k_rel_hash_collect<<<gh, kBlock, 0, s>>>(m, n, live, nid, rkey, pos);
      const size_t hs = (size_t)m.hash_mask + 1;
      VG_HIP(hipMemsetAsync(m.hkey, 0xff, hs * sizeof(uint64_t), s));
      VG_HIP(hipMemsetAsync(m.hval, 0xff, hs * sizeof(int), s));
      VG_HIP(hipMemsetAsync(m.hfirst, 0x7f, hs * sizeof(int), s));
      int* rcnt = (int*)(cnt + 16);  // the rounds' unplaced counts (in the scratch's 256-byte counter block)
      int herr_h = hcnt[kRelRootsLive] > (unsigned long long)m.hash_mask ? 1 : 0;
      constexpr int kRounds = 8;
      for (long done = 0; !herr_h && n_live > 0;) {
        VG_HIP(hipMemsetAsync(rcnt, 0, kRounds * sizeof(int), s));
        for (int t = 0; t < kRounds; t++) {
          k_rel_hash_round<<<grid_for(n_live), kBlock, 0, s>>>(m, n_live, rkey, pos, 0, rcnt + t);
          k_rel_hash_round<<<grid_for(n_live), kBlock, 0, s>>>(m, n_live, rkey, pos, 1, rcnt + t);
        }
        int left = 0;
        VG_HIP(hipMemcpyAsync(&left, rcnt + kRounds - 1, sizeof(int), hipMemcpyDeviceToHost, s));
        VG_HIP(hipStreamSynchronize(s));
        if (left == 0) break;
        done += kRounds;
        if (done > (long)m.hash_mask + 1) herr_h = 1;  // (never: each round places the lowest bidder)
      }
      if (herr_h) {
        ctx->err = "vg_release_far: root hash rebuild failed";
        return VG_E_STATE;
      }
      // the point_fix arena: the kept blocks packed in node order (read with
      // the old records' offsets, so before the records are rewritten)
      const int gn = grid_for((long)n * 64);
      k_rel_fix<<<gn, kBlock, 0, s>>>(m, n, m.fix_pnt, 3, fblk, foff, (double*)gp);
      VG_HIP(hipMemcpyAsync(m.fix_pnt, gp, (size_t)fix_new * 3 * sizeof(double), hipMemcpyDeviceToDevice, s));
      k_rel_fix<<<gn, kBlock, 0, s>>>(m, n, m.fix_var, 9, fblk, foff, (double*)gp);
      VG_HIP(hipMemcpyAsync(m.fix_var, gp, (size_t)fix_new * 9 * sizeof(double), hipMemcpyDeviceToDevice, s));
      // node ids held outside the pool
      if (nslide > 0) k_rel_remap<<<grid_for(nslide), kBlock, 0, s>>>(m.slide, nslide, n, live, nid);
      const long nwp = (long)m.cap_wp * W;
      k_rel_remap<<<grid_for(nwp), kBlock, 0, s>>>(m.wp_leaf, nwp, n, live, nid);
      // the node records (references remapped), then every other per-node array
      k_rel_hdr<<<grid_for(n), kBlock, 0, s>>>(m, n, live, nid, fblk, foff, (NodeHdr*)gp);
      VG_HIP(hipMemcpyAsync(m.hdr, gp, (size_t)n_live * sizeof(NodeHdr), hipMemcpyDeviceToDevice, s));
      struct Arr {
        void* p;
        size_t rec;  // bytes per node
        int fresh;   // byte value of a fresh record (-1: left as is, the allocation writes it)
      };
      const Arr arrs[] = {
          {m.pl, sizeof(PlaneRec), 0},          {m.pcr_add, sizeof(Clu), 0},       {m.pcr_fix, sizeof(Clu), 0},
          {m.cov_add, (size_t)kCovN * 8, 0},    {m.eig, 12 * 8, 0},                {m.jour, 8, 0},
          {m.dbox, 6 * 8, -1},                  {m.pcrs, (size_t)W * sizeof(Clu), 0}, {m.nscr, 16, 0xff},
          {m.pend, 8, -1},                      {m.cfirst, 32, 0x7f},              {m.leaf_cnt, 4, 0},
          {m.leaf_seg, 4, -1},                  {m.lseg, (size_t)W * 8, 0},        {m.stamp, 4, 0},
      };
      for (const Arr& a : arrs) {
        const int w = (int)(a.rec / 4);
        const long total = (long)n * w;
        k_rel_gather<<<grid_for(total), kBlock, 0, s>>>((const uint32_t*)a.p, (uint32_t*)gp, w, total, live, nid);
        VG_HIP(hipMemcpyAsync(a.p, gp, (size_t)n_live * a.rec, hipMemcpyDeviceToDevice, s));
        if (a.fresh >= 0 && n > n_live)
          VG_HIP(hipMemsetAsync((char*)a.p + (size_t)n_live * a.rec, a.fresh, (size_t)(n - n_live) * a.rec, s));
      }
      k_rel_gather_u8<<<grid_for(n), kBlock, 0, s>>>(m.in_slide, (uint8_t*)gp, n, live, nid);
      VG_HIP(hipMemcpyAsync(m.in_slide, gp, (size_t)n_live, hipMemcpyDeviceToDevice, s));
      if (n > n_live) VG_HIP(hipMemsetAsync(m.in_slide + n_live, 0, (size_t)(n - n_live), s));
      VG_HIP(hipMemsetAsync(ctx->wk.cand_bits, 0, (ctx->cap.max_nodes / 32 + 1) * sizeof(uint32_t), s));
      k_rel_counts<<<1, 64, 0, s>>>(m, n_live, fix_new);
      VG_HIP(hipGetLastError());
      return VG_OK;
    });
  });
  if (r != VG_OK) return r;
  (void)fix_new;
  out[0] = release ? (long long)hcnt[kRelDead] : -1;
  out[1] = (long long)hcnt[kRelNodesDead];
  out[2] = (long long)hcnt[kRelRootsLive];
  out[3] = n_live;
  out[4] = (long long)hcnt[kRelFixHeld];
  out[5] = did ? fix_new : nfix_used;
  return VG_OK;
}

// test hook (vgx_roots): every hashed root's key, jour stamp, flags and
// subtree counts, in hash-slot order; *count = the roots (rows past cap unwritten)
int map_roots(vg_ctx* ctx, long long* key, double* jour, int* flags, int* nodes, int* nfix, int cap, int* count) {
  DevMap& m = ctx->map;
  hipStream_t s = ctx->stream;
  int hc[kCntN];
  VG_HIP(hipMemcpyAsync(hc, m.counters, sizeof(hc), hipMemcpyDeviceToHost, s));
  VG_HIP(hipStreamSynchronize(s));
  const int n = hc[kCntNodes] < m.cap_nodes ? hc[kCntNodes] : m.cap_nodes;
  const size_t un = (size_t)(n > 0 ? n : 1);
  // scratch: the row count, per node (subtree nodes, point_fix), then the rows
  const size_t o_cnt = 0, o_nodes = 256, o_fix = o_nodes + un * 4, o_key = ((o_fix + un * 4 + 255) / 256) * 256,
               o_jour = o_key + un * 24, o_flags = o_jour + un * 8, o_on = o_flags + un * 4, o_of = o_on + un * 4,
               total = o_of + un * 4;
  void* sp = nullptr;
  int nr = 0;
  const int r = with_scratch(ctx, total, &sp, [&]() -> int {
    char* b = (char*)sp;
    VG_HIP(hipMemsetAsync(b, 0, o_key, s));
    if (n > 0) {
      k_roots_count<<<grid_for(n), kBlock, 0, s>>>(m, n, (int*)(b + o_nodes), (int*)(b + o_fix));
      k_roots_rows<<<grid_for((long)m.hash_mask + 1), kBlock, 0, s>>>(
          m, n, (int*)(b + o_nodes), (int*)(b + o_fix), (int*)(b + o_cnt), (long long*)(b + o_key),
          (double*)(b + o_jour), (int*)(b + o_flags), (int*)(b + o_on), (int*)(b + o_of));
    }
    VG_HIP(hipGetLastError());
    VG_HIP(hipMemcpyAsync(&nr, b + o_cnt, sizeof(int), hipMemcpyDeviceToHost, s));
    VG_HIP(hipStreamSynchronize(s));
    const int k = nr < cap ? nr : cap;
    if (k > 0 && key) {
      VG_HIP(hipMemcpyAsync(key, b + o_key, (size_t)k * 24, hipMemcpyDeviceToHost, s));
      VG_HIP(hipMemcpyAsync(jour, b + o_jour, (size_t)k * 8, hipMemcpyDeviceToHost, s));
      VG_HIP(hipMemcpyAsync(flags, b + o_flags, (size_t)k * 4, hipMemcpyDeviceToHost, s));
      VG_HIP(hipMemcpyAsync(nodes, b + o_on, (size_t)k * 4, hipMemcpyDeviceToHost, s));
      VG_HIP(hipMemcpyAsync(nfix, b + o_of, (size_t)k * 4, hipMemcpyDeviceToHost, s));
    }
    return VG_OK;
  });
  if (r != VG_OK) return r;
  *count = nr;
  return VG_OK;
}

}  // namespace vg
