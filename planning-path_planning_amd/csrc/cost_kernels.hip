// cost_kernels.hip -- computeCostMap pre-pass on the device:
// reference src/DyMu_GlobalPathPlanning.cpp:145-181 (computeCostMap),
// :186-210 (calculateSlope), :217-293 (calculateNominalCost), :297-308
// (smoothCost), with quirks Q1-Q4, plus the per-node speed of :527-528.
//
// Two elementwise/stencil kernels over the row-major SoA planner state (pitch
// ld); one thread per cell, 2-D grid-stride (rows on blockIdx.y, columns on
// blockIdx.x), coalesced along rows and free of 64-bit index division.
//   k_cost_nominal: terrain class (border -> 0), slope (3x3 central /
//     one-sided differences), nominal cost from the LUT, sticky obstacle flag,
//     locomotion mode, hazard/trafficability of obstacles.
//   k_cost_smooth: cost = (previous cost + sum of the nb4 raw costs) / (1 + #nb4)
//     (Q1), optionally fused with the speed packing F = (res*cost)*((2+hd)-tr).
// Built with -ffp-contract=off: every operation rounds like the host code.
// atan is the device libm's (ocml), which may differ from glibc's in the last
// ulp; parity is therefore stated with a tolerance.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fim_kernels.h"

namespace dymu {

namespace {

__device__ __forceinline__ double slope_at(const double* E, int64_t ld, uint32_t nx, uint32_t ny,
                                           uint32_t i, uint32_t j, double res) {
  const int64_t k = (int64_t)j * ld + i;
  double dx, dy;
  if (i == 0)
    dx = (E[k + 1] - E[k]) / res;
  else if (i == nx - 1)
    dx = (E[k] - E[k - 1]) / res;
  else
    dx = (E[k + 1] - E[k - 1]) * 0.5 / res;
  if (j == 0)
    dy = (E[k + ld] - E[k]) / res;
  else if (j == ny - 1)
    dy = (E[k] - E[k - ld]) / res;
  else
    dy = (E[k + ld] - E[k - ld]) * 0.5 / res;
  return atan(sqrt(dx * dx + dy * dy));
}

// rows j on blockIdx.y, columns i on blockIdx.x (both grid-strided)
#define DYMU_FOR_CELLS(a)                                                             \
  for (uint32_t j = blockIdx.y; j < (a).ny; j += gridDim.y)                           \
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (a).nx;              \
         i += gridDim.x * blockDim.x)

__global__ void k_cost_nominal(CostArgs a) {
  const double kPi = 3.14159265358979323846;  // M_PI
  DYMU_FOR_CELLS(a) {
    const int64_t k = (int64_t)j * a.ld + i;
    // :162-163 border cells are terrain 0 (obstacle)
    const uint32_t t = (i == 0 || j == 0 || i == a.nx - 1 || j == a.ny - 1)
                           ? 0u
                           : (uint32_t)a.terrain_map[k];
    a.st.terrain[k] = t;
    // nx or ny == 1 has no neighbour on that axis in the reference either
    // (:186-210 reads NULL); such grids are rejected on the host.
    const double sl = slope_at(a.elevation, a.ld, a.nx, a.ny, i, j, a.res);
    a.st.slope[k] = sl;
    double raw = 0.0;  // :171 raw_cost reset
    bool obst = a.st.is_obstacle[k] != 0;
    int32_t mode = a.st.loc_mode[k];
    if (t == 0) {  // :224-234
      raw = a.cmax;
      obst = true;
    } else if ((uint64_t)(t + 1) * a.n_slopes * a.n_locs > (uint64_t)a.lut_len) {
      // terrain class beyond the LUT: the reference reads out of bounds (UB);
      // here the cell becomes an obstacle
      raw = a.cmax;
      obst = true;
    } else if (a.n_slopes == 1) {  // :235-244, Q4: terrain*numLocs + i
      double cdef = a.lut[t * a.n_locs];
      for (int m = 0; m < a.n_locs; ++m) {
        const double cc = a.lut[t * a.n_locs + m];
        if (cc < cdef) cdef = cc;
      }
      raw = raw > cdef ? raw : cdef;
    } else {  // :245-292
      const double si = sl * 180 / kPi / (a.slope_hi - a.slope_lo) * (double)(a.n_slopes - 1);
      if (si > (double)(a.n_slopes - 1)) {
        raw = a.cmax;
        obst = true;
      } else {
        const double smin = floor(si), smax = ceil(si);
        double cdef = a.cmax;
        if (a.n_locs > 1) {
          for (int m = 1; m < a.n_locs; ++m) {  // Q2: mode 0 ignored
            const double c1 = a.lut[t * a.n_slopes * a.n_locs + m * a.n_slopes + (int)smin];
            const double c2 = a.lut[t * a.n_slopes * a.n_locs + m * a.n_slopes + (int)smax];
            const double cc = c1 + (c2 - c1) * (si - smin);
            if (cc < cdef) {
              cdef = cc;
              raw = raw > cdef ? raw : cdef;
              mode = m;
            }
          }
        } else {
          const double c1 = a.lut[t * a.n_slopes + (int)smin];
          const double c2 = a.lut[t * a.n_slopes + (int)smax];
          cdef = c1 + (c2 - c1) * (si - smin);
          raw = raw > cdef ? raw : cdef;
          mode = 0;
        }
      }
    }
    a.st.raw_cost[k] = raw;
    a.st.loc_mode[k] = mode;
    if (obst) {  // isObstacle is sticky; obstacles: trafficability 0, hazard 1
      a.st.is_obstacle[k] = 1;
      a.st.traff[k] = 0.0;
      a.st.hazard[k] = 1.0;
    }
  }
}

__device__ __forceinline__ double speed(double res, double cost, double hd, double tr, bool obst) {
  return obst ? __builtin_inf() : res * cost * (2 + hd - tr);  // :527-528
}

__global__ void k_cost_smooth(CostArgs a) {
  DYMU_FOR_CELLS(a) {
    const int64_t k = (int64_t)j * a.ld + i;
    const double* R = a.st.raw_cost;
    double csum = a.st.cost[k], nn = 5;  // Q1: starts from the previous cost
    if (j == 0) nn--; else csum += R[k - a.ld];
    if (i == 0) nn--; else csum += R[k - 1];
    if (i == a.nx - 1) nn--; else csum += R[k + 1];
    if (j == a.ny - 1) nn--; else csum += R[k + a.ld];
    const double cost = csum / nn;
    a.st.cost[k] = cost;
    if (a.F) a.F[k] = speed(a.res, cost, a.st.hazard[k], a.st.traff[k], a.st.is_obstacle[k] != 0);
  }
}

__global__ void k_pack_speed(CostArgs a) {
  DYMU_FOR_CELLS(a) {
    const int64_t k = (int64_t)j * a.ld + i;
    a.F[k] = speed(a.res, a.st.cost[k], a.st.hazard[k], a.st.traff[k], a.st.is_obstacle[k] != 0);
  }
}

// 256-thread rows of workgroups: enough column blocks to cover a row, rows
// until ~8192 workgroups (32 per CU), grid-stride beyond
dim3 grid_for(uint32_t nx, uint32_t ny) {
  const uint32_t gx = nx ? (nx + 255) / 256 : 1u;
  uint32_t gy = 8192u / gx;
  if (gy < 1) gy = 1;
  if (gy > ny) gy = ny ? ny : 1u;
  if (gy > 65535u) gy = 65535u;
  return dim3(gx, gy);
}

}  // namespace

hipError_t launch_cost_map(const CostArgs& a, hipStream_t st) {
  const dim3 g = grid_for(a.nx, a.ny);
  hipLaunchKernelGGL(k_cost_nominal, g, dim3(256), 0, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_cost_smooth, g, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_pack_speed(const CostArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_speed, grid_for(a.nx, a.ny), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace dymu
