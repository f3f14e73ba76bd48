// dymu_base.hpp -- the value types the DyMu class surface needs
// (base::Waypoint, base::Pose2D, base::samples::frame::Frame, base::Time).
//
// The reference takes them from Rock base-types (src/DyMu.hpp:17-19, Eigen
// vectors underneath).  Only position[0..2], heading and orientation of the
// poses, the geometry accessors and byte buffer of the frame, and now() /
// difference / toSeconds() of the time are used, so plain structs with the
// same member names are enough.  A Rock build defines DYMU_HAVE_ROCK_BASE and
// gets the real types instead.
#pragma once

#ifdef DYMU_HAVE_ROCK_BASE
#include <base/Time.hpp>
#include <base/Waypoint.hpp>
#include <base/samples/Frame.hpp>
#else
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace base {

struct Vec3 {
  double v[3] = {0.0, 0.0, 0.0};
  double& operator[](std::size_t k) { return v[k]; }
  const double& operator[](std::size_t k) const { return v[k]; }
};

struct Vec2 {
  double v[2] = {0.0, 0.0};
  double& operator[](std::size_t k) { return v[k]; }
  const double& operator[](std::size_t k) const { return v[k]; }
};

struct Waypoint {
  Vec3 position;
  double heading = 0.0;
  double tol_position = 0.0;
  double tol_heading = 0.0;
};

struct Pose2D {
  Vec2 position;
  double orientation = 0.0;
};

struct Time {
  int64_t microseconds = 0;
  static Time now() {
    Time t;
    t.microseconds = std::chrono::duration_cast<std::chrono::microseconds>(
                         std::chrono::system_clock::now().time_since_epoch())
                         .count();
    return t;
  }
  Time operator-(const Time& o) const {
    Time t;
    t.microseconds = microseconds - o.microseconds;
    return t;
  }
  double toSeconds() const { return (double)microseconds / 1e6; }
};

namespace samples {
namespace frame {
// A byte image: pixel (i, j) starts at image[j * getRowSize() + i * getPixelSize()]
// (the traversability map of computeLocalPlanning, src/DyMu_LocalPathRepairing.cpp:243-244).
struct Frame {
  std::vector<uint8_t> image;
  uint32_t width = 0, height = 0, pixel_size = 1, row_size = 0;
  Frame() = default;
  Frame(uint32_t w, uint32_t h, uint32_t pixel_bytes = 1)
      : image((std::size_t)w * h * pixel_bytes, 0),
        width(w),
        height(h),
        pixel_size(pixel_bytes),
        row_size(w * pixel_bytes) {}
  uint32_t getWidth() const { return width; }
  uint32_t getHeight() const { return height; }
  uint32_t getPixelSize() const { return pixel_size; }
  uint32_t getRowSize() const { return row_size; }
};
}  // namespace frame
}  // namespace samples

}  // namespace base
#endif
