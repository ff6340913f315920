// mdx_host.h -- ROS-free C++ node core over the C-ABI (include/mdx.h).
//
// The reference's caller of the hot path is MotionDetectionNode (ros/src/motion_detection_node.cpp):
// it subscribes sensor_msgs/Image on ~input_image (:63), keeps a ring of the last
// trajectory_size frames (:237-261), converts them with cv_bridge::toCvCopy(msg, "rgb8") (:271) and
// runs either runOpticalFlow (:76-92, the pair path with the motion mask -- compiled but only
// reachable from commented-out code) or runOpticalFlowTrajectory + fitSubspace (:94-110, :341-348,
// the live path), then publishes RGB8 images (publishImage, :217-223).  This header restates that
// caller without ROS or OpenCV: messages are plain structs, publishing is a callback, and every
// per-pixel step goes through libmdx.so.  No Python anywhere on this path.
#ifndef MDX_HOST_H_
#define MDX_HOST_H_

#include <cstdint>
#include <deque>
#include <fstream>
#include <functional>
#include <string>
#include <vector>

#include "mdx.h"

namespace mdx_host {

// sensor_msgs/Image, the fields the node reads
struct Image {
    uint32_t height = 0, width = 0;
    std::string encoding;          // "mono8", "rgb8" or "bgr8"
    uint32_t step = 0;             // row pitch in bytes
    std::vector<uint8_t> data;
};

// cv_bridge::toCvCopy(msg, "rgb8") (node.cpp:271): mono8 replicated to three channels, bgr8
// reordered, rows made contiguous (step = 3 * width).  Throws std::invalid_argument otherwise.
Image to_rgb8(const Image& msg);

// ROS parameters of the node that the path reads (node.cpp:29-44, :237-240, :346); defaults are the
// reference's own (egomotion true :40, min_vector_size 1.0 :44, skip_frames 1 and num_motions 2
// :238-240, sigma 0.5 :346) except pixel_step, which has no default there (:29; 10 in the launch
// files) and use_all_frames, whose constructor default (false, :37) disagrees with main()'s (true,
// :568) -- every launch file sets it true.
struct Params {
    int pixel_step = 10;
    double min_vector_size = 1.0;
    int skip_frames = 1;
    int num_motions = 2;
    bool egomotion = true;
    bool use_all_frames = true;
    double sigma = 0.5;
    // which caller body to run per frame: true = the live path (trajectories + fitSubspace,
    // node.cpp:266-348), false = runOpticalFlow on the ring's last two frames (:76-92), the only
    // caller that produces the motion mask
    bool live_path = true;
    uint32_t seed = 1;             // the reference seeds rand() with time(NULL) (outlier_detector.cpp:17)
    int subspace_precision = MDX_SUBSPACE_F64;   // or MDX_SUBSPACE_F32 (the reference's float shape)
};

// One processed frame's outputs (what the node hands to its publishers / logs).
struct FrameResult {
    int num_vectors = 0;                       // the calculator's return value
    int w = 0, h = 0, npts = 0;
    std::vector<double> vector_image;          // h * w * 4: the node's optical_flow_vectors Mat, Vec4d per
                                               // pixel, zero where no store landed (node.cpp:81 / :98)
    // pair path
    std::vector<float> next_pts;               // 2 * npts
    std::vector<uint8_t> status;               // npts
    std::vector<uint8_t> mask;                 // h * w, thresholded |warp(gray1) - gray2|
    double H[9] = {0};
    int rc = 0;                                // MDX_OK or MDX_EDEGENERATE
    // live path
    std::vector<std::vector<float>> trajectories;   // complete ones, (x, y) * traj_size each
    std::vector<float> outlier_points;              // fitSubspace's outlier_points, (x, y) each
    std::vector<int> subspace_columns;              // indices (into trajectories) of the winning sample
};

using Publisher = std::function<void(const std::string& topic, const Image& msg)>;

class MotionDetectionNode {
public:
    // device: HIP device of this camera stream's context (one context per stream / GPU)
    MotionDetectionNode(const Params& p, int device, int max_w, int max_h, Publisher pub);
    ~MotionDetectionNode();
    MotionDetectionNode(const MotionDetectionNode&) = delete;
    MotionDetectionNode& operator=(const MotionDetectionNode&) = delete;

    // imageCallback (node.cpp:235-455): returns true and fills *out when the frame was processed.
    bool image_callback(const Image& msg, FrameResult* out);

    Params& params() { return p_; }
    long global_frame_count() const { return global_frame_count_; }
    int trajectory_size() const { return p_.egomotion ? 2 * p_.num_motions + 1 : 2; }   // :241-245

private:
    void run_pair(const Image& a, const Image& b, FrameResult* r);
    void run_live(int nimg, FrameResult* r);
    void publish(const std::string& topic, const Image& img) const;

    Params p_;
    Publisher pub_;
    mdx_ctx* ctx_ = nullptr;
    mdx_rand_state rng_{};
    std::deque<Image> raw_images_;
    Image last_rgb_;                          // the newest frame as rgb8 (also in the device ring)
    bool image_received_ = false;
    long global_frame_count_ = 0;
};

// RGB8 renderings the node publishes, both under topic names of this build's own (kTopicMask,
// kTopicFlowMarkers), never under the reference's: the motion mask replicated to three channels
// (the new, optional mask topic of SURVEY.md §8b), and the frame with a CV_RGB(0, 0, 255) mark at
// each vector showOpticalFlowVectors would draw.  The reference's ~optical_flow_image carries
// anti-aliased arrows (optical_flow_visualizer.cpp:23-71, published at node.cpp:83-85, :101-103);
// its rendering is out of scope, so that topic is not published here ("Topics").
constexpr const char* kTopicMask = "motion_mask_image";
constexpr const char* kTopicFlowMarkers = "mdx_flow_markers_image";
Image mask_image(const std::vector<uint8_t>& mask, int w, int h);
Image flow_image(const Image& rgb, const std::vector<double>& vector_image, int pixel_step, double min_vector_size);

// On-disk formats: OpticalFlowCalculator::writeFlow / writeTrajectories
// (optical_flow_calculator.cpp:509-562) and MotionLogger (motion_logger.cpp:31-47), written with
// std::ofstream so the numbers format exactly as the reference's.
void write_flow(const std::vector<double>& vector_image, int w, int h, int pixel_step, const std::string& filename);
void write_trajectories(const std::vector<std::vector<float>>& trajectories, const std::string& filename);

class MotionLogger {
public:
    explicit MotionLogger(const std::string& path) : out_(path) {}
    void write_contour(const std::vector<int>& xy, int frame_number, int contour_id);
    void write_bounding_box(int x, int y, int width, int height, int frame_number, int contour_id);

private:
    std::ofstream out_;
};

}  // namespace mdx_host

#endif  // MDX_HOST_H_
