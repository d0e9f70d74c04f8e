// decode.hip — SURVEY §8(f) row f3: sensor records -> the scan the pipeline
// consumes. Replaces LidarPointCloudDecoder's handlers
// (src/sensor/lidar_pointcloud_decoder.cpp:21-240) and pcl_handler's scan
// preparation (src/sensor/lidar_decoder.cpp:7-43: sort by per-point time,
// drop the tail beyond 0.11 s, two dummy points for an empty scan).
//
// One lane per record: field decode (the reference's float / double
// conversions), the point_filter_num stride and the blind test, and a 32-bit
// order-preserving key of the float time (dropped records key to the end);
// one stable radix sort of (key, record index); one gather into SoA x, y, z,
// intensity, time. The Velodyne sweep without usable per-point times derives
// times from an unwrapped yaw with a sequential state machine (bias, cool
// down) — done on the host, as in the reference.
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <vector>

#include "vg_internal.h"

namespace vg {

__host__ __device__ __forceinline__ float rd_f32(const unsigned char* p) {
  float v;
  __builtin_memcpy(&v, p, 4);
  return v;
}
__host__ __device__ __forceinline__ double rd_f64(const unsigned char* p) {
  double v;
  __builtin_memcpy(&v, p, 8);
  return v;
}
__host__ __device__ __forceinline__ uint32_t rd_u32(const unsigned char* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}

// order-preserving map of a float onto uint32 (negative times sort first)
__device__ __forceinline__ uint32_t time_key(float t) {
  const uint32_t b = __float_as_uint(t);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// decoded record i -> SoA slot i, sort key / index; time already derived
// (velodyne yaw mode: host-computed times in htime)
__global__ void k_decode(int n, const unsigned char* __restrict__ rec, vg_lidar_format f, double t0,
                         const float* __restrict__ htime, float* __restrict__ ox, float* __restrict__ oy,
                         float* __restrict__ oz, float* __restrict__ oi, float* __restrict__ ot,
                         uint32_t* __restrict__ keys, uint32_t* __restrict__ idx, int* __restrict__ nkeep) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned char* r = rec + (size_t)i * f.stride;
    const float x = rd_f32(r + f.off_x), y = rd_f32(r + f.off_y), z = rd_f32(r + f.off_z);
    float in = 0.0f, t = 0.0f;
    bool keep;
    const bool stride_ok = (i % f.point_filter_num) == 0;
    const float d3 = (x * x + y * y) + z * z;
    switch (f.kind) {
      case VG_LIVOX:  // livox_handler 60-77
        in = (float)r[f.off_intensity];
        t = (float)((double)rd_u32(r + f.off_time) * (1e-9));
        keep = stride_ok && d3 > f.blind;
        break;
      case VG_VELODYNE:  // velodyne_handler 85-101 (time mode) / yaw mode (htime, already filtered)
        if (htime) {
          t = htime[i];
          keep = t >= 0.0f;  // the host marks dropped records negative-infinite
        } else {
          t = rd_f32(r + f.off_time);
          keep = stride_ok && d3 > f.blind;
        }
        break;
      case VG_OUSTER:  // ouster_handler 140-163
        in = rd_f32(r + f.off_intensity);
        t = (float)((double)rd_u32(r + f.off_time) / 1e9);
        keep = stride_ok && d3 > f.blind;
        break;
      case VG_HESAI:  // hesai_handler 165-194
        in = rd_f32(r + f.off_intensity);
        t = (float)(rd_f64(r + f.off_time) - t0);
        keep = stride_ok && d3 > f.blind;
        break;
      case VG_ROBOSENSE:  // robosense_handler 196-223 (blind on x, y)
        in = rd_f32(r + f.off_intensity);
        t = (float)(rd_f64(r + f.off_time) - f.time_base);
        keep = stride_ok && (x * x + y * y) > f.blind;
        break;
      default:  // tartanair_handler 225-240: every point, time 0
        keep = true;
        break;
    }
    if (keep && (double)t > 0.11) keep = false;  // lidar_decoder.cpp:32-35
    ox[i] = x;
    oy[i] = y;
    oz[i] = z;
    oi[i] = in;
    ot[i] = t;
    keys[i] = keep ? time_key(t) : 0xffffffffu;
    idx[i] = (uint32_t)i;
    if (keep) atomicAdd(nkeep, 1);
  }
}

__global__ void k_decode_gather(int m, const uint32_t* __restrict__ idx, const float* __restrict__ ix,
                                const float* __restrict__ iy, const float* __restrict__ iz,
                                const float* __restrict__ ii, const float* __restrict__ it, float* __restrict__ o) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
    const uint32_t i = idx[j];
    o[j] = ix[i];
    o[m + j] = iy[i];
    o[2 * (size_t)m + j] = iz[i];
    o[3 * (size_t)m + j] = ii[i];
    o[4 * (size_t)m + j] = it[i];
  }
}

// velodyne_handler's yaw mode (104-137): the unwrapped yaw and its cool-down
// are a running state over the sweep, so the host derives the times; records
// it drops get -inf
static void velodyne_yaw_times(const unsigned char* rec, int n, const vg_lidar_format& f, std::vector<float>& t) {
  t.assign(n, -INFINITY);
  bool first = true;
  double yaw0 = 0, yaw_last = 0, bias = 0;
  int cool = 0;
  for (int i = 0; i < n; i++) {
    const unsigned char* r = rec + (size_t)i * f.stride;
    const float x = rd_f32(r + f.off_x), y = rd_f32(r + f.off_y), z = rd_f32(r + f.off_z);
    if (std::fabs(x) < 0.1) continue;
    double yaw = std::atan2(y, x) * 57.2957795 - bias;
    if (first) {
      yaw0 = yaw_last = yaw;
      first = false;
    }
    if ((x * x + y * y) + z * z < f.blind) continue;
    if ((yaw - yaw_last) > 180 && cool-- <= 0) {
      bias += 360;
      yaw -= 360;
      cool = 1000;
    }
    if (std::fabs(yaw - yaw_last) > 180) yaw += 360;
    const float c = (float)((yaw0 - yaw) / f.omega_l);
    yaw_last = yaw;
    if (c >= 0 && c < 0.1 && (i % f.point_filter_num) == 0) t[i] = c;
  }
}

int decode_scan(vg_ctx* ctx, const void* records, int n, const vg_lidar_format* fmt, float* xyz, float* inten,
                float* time, int* n_out) {
  VG_TRY(host_sync(ctx));  // the staging buffers are shared with the pipeline
  vg_lidar_format f = *fmt;
  f.blind = fmt->blind * fmt->blind;  // node.cpp:210
  *n_out = 0;
  if (n > ctx->cap.max_points_per_scan) {
    ctx->err = "vg_decode_scan: more records than max_points_per_scan";
    return VG_E_CAPACITY;
  }
  if (f.point_filter_num <= 0 || f.stride <= 0) {
    ctx->err = "vg_decode_scan: bad format";
    return VG_E_ARG;
  }
  const unsigned char* hrec = static_cast<const unsigned char*>(records);
  int m = 0;
  std::vector<float> soa;
  if (n > 0) {
    hipStream_t s = ctx->stream;
    // device scratch: the downsample's sort buffers are idle here (host_sync)
    DownsampleBufs& d = ctx->ds;
    const size_t bytes = (size_t)n * f.stride;
    if (bytes > (size_t)ctx->cap.max_points_per_scan * 64) {
      ctx->err = "vg_decode_scan: records wider than 64 bytes";
      return VG_E_ARG;
    }
    unsigned char* drec = reinterpret_cast<unsigned char*>(ctx->wk.k0);  // >= 8 B x max_points x (W+1)
    VG_HIP(hipMemcpyAsync(drec, hrec, bytes, hipMemcpyHostToDevice, s));
    double t0 = 0.0;
    if (f.kind == VG_HESAI) t0 = rd_f64(hrec + f.off_time);  // the first record's timestamp (hesai_handler 171)
    std::vector<float> ht;
    float* dht = nullptr;
    if (f.kind == VG_VELODYNE) {
      // usable per-point times when the last one lies in (0.01, 0.12) s (88)
      const float tl = rd_f32(hrec + (size_t)(n - 1) * f.stride + f.off_time);
      if (!(tl > 0.01 && tl < 0.12)) {
        velodyne_yaw_times(hrec, n, f, ht);
        dht = reinterpret_cast<float*>(ctx->wk.u0);
        VG_HIP(hipMemcpyAsync(dht, ht.data(), (size_t)n * sizeof(float), hipMemcpyHostToDevice, s));
      }
    }
    float* sx = ctx->d_x;
    float* sy = ctx->d_y;
    float* sz = ctx->d_z;
    float* si = ctx->d_i;
    float* st = ctx->d_t;
    int* nk = d.flags + 2;
    VG_HIP(hipMemsetAsync(nk, 0, sizeof(int), s));
    k_decode<<<grid_for(n), kBlock, 0, s>>>(n, drec, f, t0, dht, sx, sy, sz, si, st, d.head, d.idx, nk);
    size_t need = 0;
    VG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, need, d.head, d.pos, d.idx, d.idx_sorted, n, 0, 32, s));
    if (need > d.tmp_bytes) {
      ctx->err = "vg_decode_scan: sort workspace too small";
      return VG_E_CAPACITY;
    }
    size_t tb = d.tmp_bytes;
    VG_HIP(hipcub::DeviceRadixSort::SortPairs(d.tmp, tb, d.head, d.pos, d.idx, d.idx_sorted, n, 0, 32, s));
    VG_HIP(hipMemcpyAsync(ctx->h_pinned, nk, sizeof(int), hipMemcpyDeviceToHost, s));
    VG_HIP(hipStreamSynchronize(s));
    m = ctx->h_pinned[0];
    if (m > 0) {
      float* o = reinterpret_cast<float*>(ctx->wk.k1);
      k_decode_gather<<<grid_for(m), kBlock, 0, s>>>(m, d.idx_sorted, sx, sy, sz, si, st, o);
      soa.resize((size_t)5 * m);
      VG_HIP(hipMemcpyAsync(soa.data(), o, soa.size() * sizeof(float), hipMemcpyDeviceToHost, s));
      VG_HIP(hipStreamSynchronize(s));
    }
    VG_HIP(hipMemsetAsync(d.flags, 0, 4 * sizeof(int), s));
    VG_HIP(hipStreamSynchronize(s));
  }
  if (m == 0) {  // lidar_decoder.cpp:16-26: two dummy points at the origin, times 0 and 0.09
    for (int k = 0; k < 2; k++) {
      xyz[3 * k] = xyz[3 * k + 1] = xyz[3 * k + 2] = 0.0f;
      if (inten) inten[k] = 0.0f;
      time[k] = k == 0 ? 0.0f : 0.09f;
    }
    *n_out = 2;
    return VG_OK;
  }
  for (int j = 0; j < m; j++) {
    xyz[3 * j] = soa[j];
    xyz[3 * j + 1] = soa[(size_t)m + j];
    xyz[3 * j + 2] = soa[2 * (size_t)m + j];
    if (inten) inten[j] = soa[3 * (size_t)m + j];
    time[j] = soa[4 * (size_t)m + j];
  }
  *n_out = m;
  return VG_OK;
}

}  // namespace vg
