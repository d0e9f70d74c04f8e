// sync.cpp — SURVEY §8(f) row f3, the replay side: sync_packages
// (src/sensor/sync.cpp:18-96) as a context-free packager. Scans (their
// header time and last point time) and IMU samples are pushed in arrival
// order; vg_sync_pop hands out one scan with the IMU samples up to its end
// time under the reference's rules: a scan waits until an IMU sample newer
// than its end has arrived, the samples taken are those stamped <= the end
// (the one that stops the scan stays queued), a package with 4 or fewer
// samples is dropped (its samples too), and the point_notime mode rebuilds
// the scan window from consecutive header times (the first scan only primes
// it). An IMU queue drained by a package is the reference's exit(0): here
// VG_E_STATE.
#include <deque>
#include <vector>

#include "vg_internal.h"

struct vg_sync {
  int point_notime = 0;
  struct Scan {
    double beg, last;
    int id;
  };
  std::deque<Scan> scans;
  std::deque<std::vector<double>> imu;  // t, gyr 3, acc 3
  double imu_last_time = -1;
  double last_pcl_time = -1;
  bool pl_ready = false;
  Scan cur{0, 0, -1};
  double beg = 0, end = 0;
};

extern "C" {

vg_sync* vg_sync_create(int point_notime) {
  vg_sync* s = new vg_sync();
  s->point_notime = point_notime;
  return s;
}

void vg_sync_destroy(vg_sync* s) { delete s; }

int vg_sync_push_scan(vg_sync* s, double header_time, double last_point_time, int scan_id) {
  if (!s) return VG_E_ARG;
  s->scans.push_back({header_time, last_point_time, scan_id});
  return VG_OK;
}

int vg_sync_push_imu(vg_sync* s, const double* imu7) {  // imu_handler (subscribers.cpp:12-20)
  if (!s || !imu7) return VG_E_ARG;
  s->imu_last_time = imu7[0];
  s->imu.emplace_back(imu7, imu7 + 7);
  return VG_OK;
}

int vg_sync_pop(vg_sync* s, int* scan_id, double* beg, double* end, double* imu7, int cap, int* m, int* ready) {
  if (!s || !scan_id || !beg || !end || !m || !ready) return VG_E_ARG;
  *ready = 0;
  *m = 0;
  if (!s->pl_ready) {  // step 1 (sync.cpp:24-58)
    if (s->scans.empty()) return VG_OK;
    s->cur = s->scans.front();
    s->scans.pop_front();
    s->beg = s->cur.beg;
    s->end = s->beg + s->cur.last;
    if (s->point_notime) {
      if (s->last_pcl_time < 0) {
        s->last_pcl_time = s->beg;
        return VG_OK;
      }
      s->end = s->beg;
      s->beg = s->last_pcl_time;
      s->last_pcl_time = s->end;
    }
    s->pl_ready = true;
  }
  if (s->imu_last_time <= s->end) return VG_OK;  // 60-63
  std::vector<double> taken;  // 66-76
  int n = 0;
  double t = s->imu.front()[0];
  while (!s->imu.empty() && t < s->end) {
    t = s->imu.front()[0];
    if (t > s->end) break;
    taken.insert(taken.end(), s->imu.front().begin(), s->imu.front().end());
    s->imu.pop_front();
    n++;
  }
  s->pl_ready = false;
  if (s->imu.empty()) return VG_E_STATE;  // 79-82: the IMU stream broke (the reference exits)
  if (n <= 4) {  // 87-94: too few samples, the scan is dropped
    *ready = -1;
    return VG_OK;
  }
  *scan_id = s->cur.id;
  *beg = s->beg;
  *end = s->end;
  *m = n;
  if (imu7)
    for (int k = 0; k < 7 * n && k < 7 * cap; k++) imu7[k] = taken[k];
  *ready = 1;
  return VG_OK;
}

}  // extern "C"
