// vina_node.cpp — ROS 2 front end of the MI355X LIO core:
// the reference node's parameters (node.cpp:52-291), subscriptions
// (node.cpp:144-170) and outputs (publishers.cpp:42-97, io.cpp:67-77) over
// vina_gpu::NodeCore (include/vina_node_core.hpp), which holds everything that
// is not message plumbing and is tested without ROS (tests/test_node_core.py).
// Built by CMakeLists.txt only when rclcpp is found (this image has no ROS).
#include <geometry_msgs/msg/transform_stamped.hpp>
#include <rclcpp/rclcpp.hpp>
#include <sensor_msgs/msg/imu.hpp>
#include <sensor_msgs/msg/point_cloud2.hpp>
#include <sensor_msgs/point_cloud2_iterator.hpp>
#include <tf2_ros/transform_broadcaster.h>
#ifdef VG_HAVE_LIVOX
#include <livox_ros_driver2/msg/custom_msg.hpp>
#endif
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <vector>
#include "vina_node_core.hpp"

namespace {

double stamp_sec(const builtin_interfaces::msg::Time& t) { return t.sec + t.nanosec * 1e-9; }

// the per-format time field of a PointCloud2 (the reference's point structs,
// lidar_pointcloud_decoder.hpp): Velodyne "time", Ouster "t", Hesai /
// RoboSense "timestamp"; TartanAir has none
const char* time_field(int kind) {
  switch (kind) {
    case VG_VELODYNE: return "time";
    case VG_OUSTER: return "t";
    case VG_HESAI:
    case VG_ROBOSENSE: return "timestamp";
    default: return nullptr;
  }
}

int field_offset(const sensor_msgs::msg::PointCloud2& m, const char* name) {
  if (!name) return -1;
  for (const auto& f : m.fields)
    if (f.name == name) return (int)f.offset;
  return -1;
}

class VinaNode : public rclcpp::Node {
 public:
  VinaNode() : rclcpp::Node("vina_slam") {
    vg_config c;
    memset(&c, 0, sizeof(c));
    const std::string lid_topic = declare_parameter("General.lid_topic", std::string("/rslidar_points"));
    const std::string imu_topic = declare_parameter("General.imu_topic", std::string("/imu"));
    kind_ = (int)declare_parameter("General.lidar_type", 0);
    const double blind = declare_parameter("General.blind", 0.1);
    const int filter_num = (int)declare_parameter("General.point_filter_num", 3);
    const std::vector<double> et = declare_parameter("General.extrinsic_tran", std::vector<double>(3, 0.0));
    const std::vector<double> er = declare_parameter("General.extrinsic_rota", std::vector<double>(9, 0.0));
    save_pose_ = declare_parameter("General.is_save_pose", 0) != 0;
    pose_file_ = declare_parameter("General.pose_save_path", std::string("")) +
                 declare_parameter("General.pose_filename", std::string("trajectory.txt"));
    c.if_BA = (int)declare_parameter("General.if_BA", 0);
    c.odo_cov_gyr = declare_parameter("Odometry.cov_gyr", 0.1);
    c.odo_cov_acc = declare_parameter("Odometry.cov_acc", 0.1);
    c.odo_rdw_gyr = declare_parameter("Odometry.rdw_gyr", 1e-4);
    c.odo_rdw_acc = declare_parameter("Odometry.rdw_acc", 1e-4);
    c.down_size = declare_parameter("Odometry.down_size", 0.1);
    c.dept_err = declare_parameter("Odometry.dept_err", 0.02);
    c.beam_err = declare_parameter("Odometry.beam_err", 0.05);
    c.voxel_size = declare_parameter("Odometry.voxel_size", 1.0);
    c.min_eigen_value = declare_parameter("Odometry.min_eigen_value", 0.0025);
    const int point_notime = (int)declare_parameter("Odometry.point_notime", 0);
    c.win_size = (int)declare_parameter("LocalBA.win_size", 10);
    c.max_layer = (int)declare_parameter("LocalBA.max_layer", 2);
    c.ba_cov_gyr = declare_parameter("LocalBA.cov_gyr", 0.1);
    c.ba_cov_acc = declare_parameter("LocalBA.cov_acc", 0.1);
    c.ba_rdw_gyr = declare_parameter("LocalBA.rdw_gyr", 1e-4);
    c.ba_rdw_acc = declare_parameter("LocalBA.rdw_acc", 1e-4);
    const std::vector<double> thre =
        declare_parameter("LocalBA.plane_eigen_value_thre", std::vector<double>(4, 1.0));
    c.imu_coef = declare_parameter("LocalBA.imu_coef", 1e-4);
    c.thread_num = (int)declare_parameter("LocalBA.thread_num", 5);
    for (int i = 0; i < 4; i++) {
      c.plane_eigen_value_thre[i] = i < (int)thre.size() ? thre[i] : 1.0;
      c.min_point[i] = (double)(i < 2 ? 20 : (i == 2 ? 15 : 10));  // node.cpp:219
    }
    for (int i = 0; i < 9; i++) c.ext_R[i] = i < (int)er.size() ? er[i] : 0.0;
    for (int i = 0; i < 3; i++) c.ext_t[i] = i < (int)et.size() ? et[i] : 0.0;
    c.max_points = 100;  // octree.cpp:70
    c.cold_start = 1;    // the node's initialization (node.cpp:293-366)
    c.scale_gravity = 0.0;  // from IMU_init (imu_ekf.cpp:181-189)

    memset(&fmt_, 0, sizeof(fmt_));
    fmt_.kind = kind_;
    fmt_.point_filter_num = filter_num;
    fmt_.blind = blind;
    fmt_.omega_l = 3610.0;
    vg_capacity cap = {0, 0, 0, 0};
    core_ = std::make_unique<vina_gpu::NodeCore>(c, &cap, fmt_, point_notime);

    rclcpp::QoS imu_qos(8000);
    imu_qos.keep_last(8000).best_effort();
    rclcpp::QoS pcl_qos(1000);
    pcl_qos.keep_last(1000).best_effort();
    sub_imu_ = create_subscription<sensor_msgs::msg::Imu>(
        imu_topic, imu_qos, [this](sensor_msgs::msg::Imu::SharedPtr m) { on_imu(*m); });
#ifdef VG_HAVE_LIVOX
    if (kind_ == VG_LIVOX)
      sub_livox_ = create_subscription<livox_ros_driver2::msg::CustomMsg>(
          lid_topic, rclcpp::SensorDataQoS(), [this](livox_ros_driver2::msg::CustomMsg::SharedPtr m) { on_livox(*m); });
    else
#endif
      sub_pcl_ = create_subscription<sensor_msgs::msg::PointCloud2>(
          lid_topic, pcl_qos, [this](sensor_msgs::msg::PointCloud2::SharedPtr m) { on_cloud(*m); });
    pub_scan_ = create_publisher<sensor_msgs::msg::PointCloud2>("/map_scan", 100);
    pub_path_ = create_publisher<sensor_msgs::msg::PointCloud2>("/map_path", 100);
    pub_cmap_ = create_publisher<sensor_msgs::msg::PointCloud2>("/map_cmap", 100);  // publishers.cpp:130
    tf_ = std::make_unique<tf2_ros::TransformBroadcaster>(*this);
  }

  ~VinaNode() override {
    if (save_pose_ && !pose_file_.empty()) core_->write_tum(pose_file_);
  }

 private:
  void on_imu(const sensor_msgs::msg::Imu& m) {
    const double g[3] = {m.angular_velocity.x, m.angular_velocity.y, m.angular_velocity.z};
    const double a[3] = {m.linear_acceleration.x, m.linear_acceleration.y, m.linear_acceleration.z};
    core_->imu(stamp_sec(m.header.stamp), g, a);
    run();
  }

  void on_cloud(const sensor_msgs::msg::PointCloud2& m) {
    vg_lidar_format f = fmt_;
    f.stride = (int)m.point_step;
    f.off_x = field_offset(m, "x");
    f.off_y = field_offset(m, "y");
    f.off_z = field_offset(m, "z");
    f.off_intensity = field_offset(m, "intensity");
    f.off_time = field_offset(m, time_field(kind_));
    f.time_base = stamp_sec(m.header.stamp);  // RoboSense stamps are absolute
    core_->scan(stamp_sec(m.header.stamp), m.data.data(), (int)(m.width * m.height), &f);
    run();
  }

#ifdef VG_HAVE_LIVOX
  // CustomPoint -> the packed record layout the decoder reads (offset_time
  // u32, x, y, z f32, reflectivity, tag, line u8, pad: 20 bytes)
  void on_livox(const livox_ros_driver2::msg::CustomMsg& m) {
    std::vector<unsigned char> rec(m.points.size() * 20, 0);
    for (size_t i = 0; i < m.points.size(); i++) {
      unsigned char* r = &rec[20 * i];
      const auto& p = m.points[i];
      const uint32_t t = p.offset_time;
      const float xyz[3] = {p.x, p.y, p.z};
      memcpy(r, &t, 4);
      memcpy(r + 4, xyz, 12);
      r[16] = p.reflectivity;
      r[17] = p.tag;
      r[18] = p.line;
    }
    vg_lidar_format f = fmt_;
    f.stride = 20;
    f.off_time = 0;
    f.off_x = 4;
    f.off_y = 8;
    f.off_z = 12;
    f.off_intensity = 16;
    core_->scan(stamp_sec(m.header.stamp), rec.data(), (int)m.points.size(), &f);
    run();
  }
#endif

  // sync_packages + the estimator; then the outputs of every scan the device
  // has finished (NodeCore::poll, no drain): the TF per new path point
  // (pub_odom_func), the path (pub_localtraj / pub_localmap re-write), and —
  // only while someone subscribes, since reading them completes the queued
  // work — the last scan in the world (/map_scan) and /map_cmap
  void run() {
    const int stepped = core_->spin();
    const bool changed = core_->poll();
    if (stepped == 0 && !changed) return;
    const auto& path = core_->path();
    if (path.size() < published_) published_ = 0;  // system_reset cleared pcl_path
    for (; published_ < path.size(); published_++) {
      const vina_gpu::PoseStamped& s = path[published_];
      geometry_msgs::msg::TransformStamped t;
      t.header.stamp = now();
      t.header.frame_id = "camera_init";
      t.child_frame_id = "aft_mapped";
      t.transform.translation.x = s.p[0];
      t.transform.translation.y = s.p[1];
      t.transform.translation.z = s.p[2];
      t.transform.rotation.x = s.q[0];
      t.transform.rotation.y = s.q[1];
      t.transform.rotation.z = s.q[2];
      t.transform.rotation.w = s.q[3];
      tf_->sendTransform(t);
    }
    if (changed) {
      path_xyz_.resize(3 * path.size());
      for (size_t i = 0; i < path.size(); i++)
        for (int k = 0; k < 3; k++) path_xyz_[3 * i + k] = (float)path[i].p[k];
      publish_xyz(pub_path_, path_xyz_);
    }
    if (stepped > 0 && pub_scan_->get_subscription_count() > 0) publish_xyz(pub_scan_, core_->scan_world());
    const bool want_cmap = pub_cmap_->get_subscription_count() > 0;
    if (want_cmap != cmap_on_) {
      core_->enable_local_map(want_cmap);
      cmap_on_ = want_cmap;
    }
    if (cmap_on_ && stepped > 0) {
      const std::vector<float> c = core_->local_map();
      std::vector<float> xyz;
      xyz.reserve(c.size() / 4 * 3);
      for (size_t i = 0; i < c.size() / 4; i++)
        for (int k = 0; k < 3; k++) xyz.push_back(c[4 * i + k]);
      publish_xyz(pub_cmap_, xyz);
    }
  }

  void publish_xyz(const rclcpp::Publisher<sensor_msgs::msg::PointCloud2>::SharedPtr& pub,
                   const std::vector<float>& xyz) {
    sensor_msgs::msg::PointCloud2 m;
    m.header.stamp = now();
    m.header.frame_id = "camera_init";  // publishers.cpp pub_pl_func
    sensor_msgs::PointCloud2Modifier mod(m);
    mod.setPointCloud2FieldsByString(1, "xyz");
    mod.resize(xyz.size() / 3);
    sensor_msgs::PointCloud2Iterator<float> x(m, "x"), y(m, "y"), z(m, "z");
    for (size_t i = 0; i < xyz.size() / 3; i++, ++x, ++y, ++z) {
      *x = xyz[3 * i];
      *y = xyz[3 * i + 1];
      *z = xyz[3 * i + 2];
    }
    pub->publish(m);
  }

  int kind_ = 0;
  vg_lidar_format fmt_;
  bool save_pose_ = false;
  std::string pose_file_;
  size_t published_ = 0;
  std::unique_ptr<vina_gpu::NodeCore> core_;
  std::unique_ptr<tf2_ros::TransformBroadcaster> tf_;
  rclcpp::Subscription<sensor_msgs::msg::Imu>::SharedPtr sub_imu_;
  rclcpp::Subscription<sensor_msgs::msg::PointCloud2>::SharedPtr sub_pcl_;
#ifdef VG_HAVE_LIVOX
  rclcpp::Subscription<livox_ros_driver2::msg::CustomMsg>::SharedPtr sub_livox_;
#endif
  rclcpp::Publisher<sensor_msgs::msg::PointCloud2>::SharedPtr pub_scan_, pub_path_, pub_cmap_;
  std::vector<float> path_xyz_;
  bool cmap_on_ = false;
};

}  // namespace

int main(int argc, char** argv) {
  rclcpp::init(argc, argv);
  rclcpp::spin(std::make_shared<VinaNode>());
  rclcpp::shutdown();
  return 0;
}
