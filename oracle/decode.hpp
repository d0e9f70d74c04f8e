// decode.hpp — TEST INFRASTRUCTURE (oracle). CPU restatement of the sensor
// decoders (src/sensor/lidar_pointcloud_decoder.cpp:21-240) and pcl_handler's
// scan preparation (src/sensor/lidar_decoder.cpp:7-43), SURVEY §8(f) row f3,
// over little-endian records described like vg_lidar_format. Sequential,
// std::sort by time as the reference (its order among equal times is the
// library's; the device path sorts stably).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace orc {

struct DecFormat {
  int kind, stride, off_x, off_y, off_z, off_intensity, off_time, point_filter_num;
  double blind, omega_l, time_base;
};
struct DecPoint {
  float x, y, z, intensity, curvature;
};

template <class T>
inline T dec_field(const unsigned char* p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}

inline std::vector<DecPoint> decode_records(const unsigned char* rec, int n, const DecFormat& fmt) {
  const double blind = fmt.blind * fmt.blind;  // node.cpp:210
  std::vector<DecPoint> out;
  auto at = [&](int i) { return rec + (size_t)i * fmt.stride; };
  auto xyz = [&](int i, DecPoint& p) {
    p.x = dec_field<float>(at(i) + fmt.off_x);
    p.y = dec_field<float>(at(i) + fmt.off_y);
    p.z = dec_field<float>(at(i) + fmt.off_z);
    p.intensity = 0.f;
    p.curvature = 0.f;
  };
  auto far = [&](const DecPoint& p) { return (p.x * p.x + p.y * p.y + p.z * p.z) > blind; };
  switch (fmt.kind) {
    case 0:  // livox_handler 60-77
      for (int i = 0; i < n; i++) {
        DecPoint p;
        xyz(i, p);
        p.intensity = (float)at(i)[fmt.off_intensity];
        p.curvature = (float)(dec_field<uint32_t>(at(i) + fmt.off_time) * (1e-9));
        if ((i % fmt.point_filter_num) == 0 && far(p)) out.push_back(p);
      }
      break;
    case 1: {  // velodyne_handler 78-138
      if (n == 0) break;
      const float tl = dec_field<float>(at(n - 1) + fmt.off_time);
      if (tl > 0.01 && tl < 0.12) {
        for (int i = 0; i < n; i++) {
          DecPoint p;
          xyz(i, p);
          p.curvature = dec_field<float>(at(i) + fmt.off_time);
          if ((i % fmt.point_filter_num) == 0 && far(p)) out.push_back(p);
        }
      } else {
        bool first = true;
        double yaw0 = 0, yaw_last = 0, bias = 0;
        int cool = 0;
        for (int i = 0; i < n; i++) {
          DecPoint p;
          xyz(i, p);
          if (std::fabs(p.x) < 0.1) continue;
          double yaw = std::atan2(p.y, p.x) * 57.2957795 - bias;
          if (first) {
            yaw0 = yaw_last = yaw;
            first = false;
          }
          if (p.x * p.x + p.y * p.y + p.z * p.z < blind) continue;
          if ((yaw - yaw_last) > 180 && cool-- <= 0) {
            bias += 360;
            yaw -= 360;
            cool = 1000;
          }
          if (std::fabs(yaw - yaw_last) > 180) yaw += 360;
          p.curvature = (float)((yaw0 - yaw) / fmt.omega_l);
          yaw_last = yaw;
          if (p.curvature >= 0 && p.curvature < 0.1 && (i % fmt.point_filter_num) == 0) out.push_back(p);
        }
      }
      break;
    }
    case 2:  // ouster_handler 140-163
      for (int i = 0; i < n; i++) {
        DecPoint p;
        xyz(i, p);
        p.intensity = dec_field<float>(at(i) + fmt.off_intensity);
        p.curvature = (float)(dec_field<uint32_t>(at(i) + fmt.off_time) / 1e9);
        if ((i % fmt.point_filter_num) == 0 && far(p)) out.push_back(p);
      }
      break;
    case 3: {  // hesai_handler 165-194
      if (n == 0) break;
      const double t0 = dec_field<double>(at(0) + fmt.off_time);
      for (int i = 0; i < n; i++) {
        DecPoint p;
        xyz(i, p);
        p.intensity = dec_field<float>(at(i) + fmt.off_intensity);
        p.curvature = (float)(dec_field<double>(at(i) + fmt.off_time) - t0);
        if ((i % fmt.point_filter_num) == 0 && far(p)) out.push_back(p);
      }
      break;
    }
    case 4:  // robosense_handler 196-223
      for (int i = 0; i < n; i++) {
        DecPoint p;
        xyz(i, p);
        p.intensity = dec_field<float>(at(i) + fmt.off_intensity);
        p.curvature = (float)(dec_field<double>(at(i) + fmt.off_time) - fmt.time_base);
        if (((i % fmt.point_filter_num) == 0) && ((p.x * p.x + p.y * p.y) > blind)) out.push_back(p);
      }
      break;
    default:  // tartanair_handler 225-240
      for (int i = 0; i < n; i++) {
        DecPoint p;
        xyz(i, p);
        out.push_back(p);
      }
  }
  // pcl_handler (lidar_decoder.cpp:16-35)
  if (out.empty()) {
    DecPoint a{0.f, 0.f, 0.f, 0.f, 0.f};
    out.push_back(a);
    a.curvature = 0.09f;
    out.push_back(a);
  }
  std::sort(out.begin(), out.end(), [](const DecPoint& a, const DecPoint& b) { return a.curvature < b.curvature; });
  while (!out.empty() && out.back().curvature > 0.11) out.pop_back();  // (the reference assumes non-empty)
  return out;
}

}  // namespace orc
