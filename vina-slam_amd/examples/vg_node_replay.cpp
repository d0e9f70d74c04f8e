// vg_node_replay — runs a recorded sensor event log through vina_gpu::NodeCore,
// the ROS-free core of the reference's ROS 2 node (include/vina_node_core.hpp,
// SURVEY rows f3/f4): IMU samples and raw LiDAR messages in arrival order, as
// the node's subscriptions would deliver them (node.cpp:153-170), each
// followed by a spin of sync_packages + the estimator. Writes the TUM pose file
// of save_pose_tum (io.cpp:67-77) and prints one summary line.
//
// Event log (little-endian):
//   "VGEVENT1" | vg_config (sizeof) | vg_lidar_format (sizeof) | int32 point_notime
//   | int32 has_seed | double seed[VG_STATE_LEN] if has_seed
//   then events: int32 type; 0: double imu[7] (t, gyr 3, acc 3);
//                1: double header_time, int32 n, int32 stride, n*stride record bytes;
//                -1 or end of file: done
//
// usage: vg_node_replay <events.bin> <out_tum.txt> [device]
#include <cstdio>
#include <cstring>
#include <vector>
#include "../../include/vina_node_core.hpp"

static bool rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s events.bin out_tum.txt [device [out_path.txt [out_cmap.bin]]]\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) {
    perror("events");
    return 1;
  }
  char magic[8];
  vg_config cfg;
  vg_lidar_format fmt;
  int point_notime = 0, has_seed = 0;
  double seed[VG_STATE_LEN];
  if (!rd(f, magic, 8) || memcmp(magic, "VGEVENT1", 8) != 0 || !rd(f, &cfg, sizeof(cfg)) ||
      !rd(f, &fmt, sizeof(fmt)) || !rd(f, &point_notime, 4) || !rd(f, &has_seed, 4) ||
      (has_seed && !rd(f, seed, sizeof(seed)))) {
    fprintf(stderr, "bad event log header\n");
    return 1;
  }
  try {
    vg_capacity cap = {0, 0, 0, 0};
    cap.max_points_per_scan = 400000;
    vina_gpu::NodeCore node(cfg, &cap, fmt, point_notime, argc > 3 ? atoi(argv[3]) : 0);
    if (has_seed) node.lio().seed(seed);
    if (argc > 5) node.enable_local_map(true);  // /map_cmap after every window BA
    std::vector<unsigned char> rec;
    int n_imu = 0, n_msg = 0, n_step = 0;
    for (;;) {
      int type = -1;
      if (!rd(f, &type, 4) || type < 0) break;
      if (type == 0) {
        double s[7];
        if (!rd(f, s, sizeof(s))) break;
        node.imu(s[0], s + 1, s + 4);
        n_imu++;
      } else {
        double stamp;
        int n, stride;
        if (!rd(f, &stamp, 8) || !rd(f, &n, 4) || !rd(f, &stride, 4) || n < 0 || stride <= 0) break;
        rec.resize((size_t)n * stride);
        if (!rd(f, rec.data(), rec.size())) break;
        node.scan(stamp, rec.data(), n);
        n_msg++;
      }
      n_step += node.spin();
    }
    const std::vector<float> w = node.scan_world();
    if (!node.write_tum(argv[2])) {
      perror("tum");
      return 1;
    }
    if (argc > 4) {  // pcl_path after the run: t x y z jour per row (the BA re-writes included)
      FILE* fp = fopen(argv[4], "w");
      if (!fp) {
        perror("path");
        return 1;
      }
      for (const vina_gpu::PoseStamped& s : node.path())
        fprintf(fp, "%.9f %.12f %.12f %.12f %.12f\n", s.t, s.p[0], s.p[1], s.p[2], s.jour);
      fclose(fp);
    }
    size_t ncmap = 0;
    if (argc > 5) {  // the last /map_cmap cloud, float32 x y z intensity
      const std::vector<float> c = node.local_map();
      ncmap = c.size() / 4;
      FILE* fc = fopen(argv[5], "wb");
      if (!fc || fwrite(c.data(), sizeof(float), c.size(), fc) != c.size()) {
        perror("cmap");
        return 1;
      }
      fclose(fc);
    }
    printf("{\"imu\": %d, \"scans\": %d, \"stepped\": %d, \"poses\": %zu, \"path\": %zu, "
           "\"last_scan_world_points\": %zu, \"cmap_points\": %zu}\n",
           n_imu, n_msg, n_step, node.tum_rows().size(), node.path().size(), w.size() / 3, ncmap);
  } catch (const vina_gpu::Error& e) {
    fprintf(stderr, "vg_node_replay: %s (code %d)\n", e.what(), e.code);
    return 1;
  }
  fclose(f);
  return 0;
}
