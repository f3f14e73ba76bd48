// dymu_base.hpp -- the value types the DyMu class surface needs
// (base::Waypoint, base::Pose2D).
//
// The reference takes them from Rock base-types (src/DyMu.hpp:17-19, Eigen
// vectors underneath).  Only position[0..2], heading and
// orientation are read or written on the global path, so a plain struct with
// the same member names is enough.  A Rock build defines
// DYMU_HAVE_ROCK_BASE and gets the real types instead.
#pragma once

#ifdef DYMU_HAVE_ROCK_BASE
#include <base/Waypoint.hpp>
#else
#include <cstddef>

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

}  // namespace base
#endif
