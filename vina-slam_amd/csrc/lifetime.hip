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
    for (int k = 0; k < 8; k++) {
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

// the kept roots' (key, new id) pairs, then the table is cleared and refilled
__global__ void __launch_bounds__(256) k_rel_hash_collect(DevMap m, int n, const int* __restrict__ live,
                                                          const int* __restrict__ nid, uint64_t* __restrict__ keys,
                                                          int* __restrict__ ids, unsigned long long* __restrict__ cnt) {
  const int hs = m.hash_mask + 1;
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < hs; s += gridDim.x * blockDim.x) {
    const uint64_t key = m.hkey[s];
    if (key == kKeyEmpty) continue;
    const int r = m.hval[s];
    if (r < 0 || r >= n || !live[r]) continue;
    const int q = (int)atomicAdd(&cnt[kRelKeys], 1ull);
    keys[q] = key;
    ids[q] = nid[r];
  }
}
__global__ void __launch_bounds__(256) k_rel_hash_fill(DevMap m, int nk, const uint64_t* __restrict__ keys,
                                                       const int* __restrict__ ids, int* __restrict__ err) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nk; q += gridDim.x * blockDim.x) {
    bool fresh = false;
    const int s = hash_insert(m.hkey, m.hash_mask, keys[q], fresh);
    if (s < 0 || !fresh) {
      atomicOr(err, 1);
      continue;
    }
    m.hval[s] = ids[q];
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
                                    (size_t)(hcnt[kRelRootsLive] + 1) * 16});
    void* gp = nullptr;
    return with_scratch(ctx, gbytes, &gp, [&]() -> int {
      // the root hash, rebuilt from the kept roots under their new ids
      auto* keys = (uint64_t*)gp;
      int* ids = (int*)(keys + hcnt[kRelRootsLive] + 1);
      const int gh = grid_for((long)m.hash_mask + 1);
      VG_HIP(hipMemsetAsync(&cnt[kRelKeys], 0, sizeof(unsigned long long), s));
      k_rel_hash_collect<<<gh, kBlock, 0, s>>>(m, n, live, nid, keys, ids, cnt);
      const size_t hs = (size_t)m.hash_mask + 1;
      VG_HIP(hipMemsetAsync(m.hkey, 0xff, hs * sizeof(uint64_t), s));
      VG_HIP(hipMemsetAsync(m.hval, 0xff, hs * sizeof(int), s));
      VG_HIP(hipMemsetAsync(m.hfirst, 0x7f, hs * sizeof(int), s));
      int* herr = (int*)&cnt[kRelN - 1];
      VG_HIP(hipMemsetAsync(herr, 0, sizeof(int), s));
      const int nk = (int)hcnt[kRelRootsLive];
      if (nk > 0) k_rel_hash_fill<<<grid_for(nk), kBlock, 0, s>>>(m, nk, keys, ids, herr);
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
      int herr_h = 0;
      VG_HIP(hipMemcpyAsync(&herr_h, herr, sizeof(int), hipMemcpyDeviceToHost, s));
      VG_HIP(hipStreamSynchronize(s));
      if (herr_h) {
        ctx->err = "vg_release_far: root hash rebuild failed";
        return VG_E_STATE;
      }
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

}  // namespace vg
