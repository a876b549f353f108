/*
 * MAM3SLAM host API — plain value types standing in for the OpenCV / Sophus / Eigen types the reference's
 * hot-path signatures use. Layouts are chosen so a maintainer can reinterpret the reference's own objects
 * without copies:
 *   KeyPoint  == cv::KeyPoint (28 bytes: pt, size, angle, response, octave, class_id)
 *   ImageView == a CV_8UC1 cv::Mat header (data, cols, rows, step)
 *   Mat8U     == an owned CV_8U matrix (descriptors N x 32, pyramid levels)
 *   SE3f      == Sophus::SE3f (unit quaternion x, y, z, w + translation)
 */
#ifndef MAM3SLAM_TYPES_H
#define MAM3SLAM_TYPES_H

#include <cstddef>
#include <cstdint>
#include <vector>

#include "../mam_match.h"
#include "../mam_orb.h"

namespace MAM3SLAM {

/* The HIP device that the calling thread's ORBmatcher / Optimizer calls run on (their device contexts are per
 * thread). One agent per GPU: each of an agent's threads (Tracking, LocalMapping) calls SetDevice(g) once.
 * Default 0. Changing it releases the thread's contexts on the old device. */
void SetDevice(int device);
int GetDevice();

struct Point2f {
    float x = 0.f, y = 0.f;
};

struct KeyPoint {
    Point2f pt;
    float size = 0.f, angle = -1.f, response = 0.f;
    int octave = 0, class_id = -1;
};
static_assert(sizeof(KeyPoint) == sizeof(mam_keypoint), "KeyPoint must match the C-ABI / cv::KeyPoint layout");

struct ImageView {
    const uint8_t* data = nullptr;
    int cols = 0, rows = 0;
    size_t step = 0;
    ImageView() = default;
    ImageView(const uint8_t* d, int c, int r, size_t s = 0) : data(d), cols(c), rows(r), step(s ? s : (size_t)c) {}
    bool empty() const { return data == nullptr || cols <= 0 || rows <= 0; }
};

struct Mat8U {
    int rows = 0, cols = 0;
    std::vector<uint8_t> data;
    void create(int r, int c) { rows = r; cols = c; data.assign((size_t)r * (size_t)c, 0); }
    bool empty() const { return rows == 0 || cols == 0; }
    uint8_t* ptr(int r) { return data.data() + (size_t)r * (size_t)cols; }
    const uint8_t* ptr(int r) const { return data.data() + (size_t)r * (size_t)cols; }
    ImageView view() const { return ImageView(data.data(), cols, rows, (size_t)cols); }
};

/* Sophus::SE3f: x_c = R(q) x_w + t. Rotation matrices use Eigen's Quaternion::toRotationMatrix formula. */
struct SE3f {
    float q[4] = {0.f, 0.f, 0.f, 1.f};
    float t[3] = {0.f, 0.f, 0.f};
    void rotationMatrix(float R[9]) const;
    SE3f inverse() const;
    SE3f operator*(const SE3f& o) const;
    void map(const float p[3], float out[3]) const;   /* R p + t */
    mam_pose toC() const;
};

/* Pinhole camera (GeometricCamera::mvParameters = fx, fy, cx, cy as float; src/CameraModels/Pinhole.cpp). */
struct Pinhole {
    float mvParameters[4] = {0.f, 0.f, 0.f, 0.f};
    Pinhole() = default;
    Pinhole(float fx, float fy, float cx, float cy) : mvParameters{fx, fy, cx, cy} {}
    void project(const float p3[3], float uv[2]) const;    /* Pinhole.cpp:35-41 */
    void toK(float K[9]) const;                            /* Pinhole.cpp:100-104 */
    mam_pinhole toC() const { return mam_pinhole{mvParameters[0], mvParameters[1], mvParameters[2], mvParameters[3]}; }
};

}  // namespace MAM3SLAM
#endif
