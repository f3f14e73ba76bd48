/*
 * engine_stub.c -- TEST DOUBLE for the sanitizer build of the host code
 * (tests/test_sanitize.py).  The HIP engine (libdymu_fim.so) cannot be loaded
 * into an AddressSanitizer process without a GPU runtime, so the host planner
 * is linked against this stub instead: every engine call fails with
 * DYMU_ERR_NO_DEVICE, which is what the real engine returns on a machine
 * without a HIP device.  Never part of the product.
 */
#include <stddef.h>
#include <stdint.h>

#include "dymu_fim.h"

#define NODEV return DYMU_ERR_NO_DEVICE

int dymu_create(dymu_ctx** out, const dymu_opts* o) { (void)o; if (out) *out = NULL; NODEV; }
int dymu_destroy(dymu_ctx* c) { (void)c; return DYMU_OK; }
const char* dymu_strerror(int rc) { (void)rc; return "no HIP device (sanitizer stub)"; }
const char* dymu_last_error(dymu_ctx* c) { (void)c; return "no HIP device (sanitizer stub)"; }
int dymu_device_alloc(dymu_ctx* c, size_t n, void** p) { (void)c; (void)n; (void)p; NODEV; }
int dymu_device_free(dymu_ctx* c, void* p) { (void)c; (void)p; NODEV; }
int dymu_host_register(dymu_ctx* c, void* p, size_t n) { (void)c; (void)p; (void)n; NODEV; }
int dymu_host_unregister(dymu_ctx* c, void* p) { (void)c; (void)p; NODEV; }
int dymu_memcpy_d2h(dymu_ctx* c, void* d, const void* s, size_t n) { (void)c; (void)d; (void)s; (void)n; NODEV; }
int dymu_memcpy_h2d(dymu_ctx* c, void* d, const void* s, size_t n) { (void)c; (void)d; (void)s; (void)n; NODEV; }
int dymu_memcpy2d_d2h(dymu_ctx* c, void* d, size_t dp, const void* s, size_t sp, size_t w, size_t h) {
  (void)c; (void)d; (void)dp; (void)s; (void)sp; (void)w; (void)h; NODEV;
}
int dymu_solve_device(dymu_ctx* c, const double* F, double* T, uint32_t nx, uint32_t ny, uint64_t ld,
                      uint32_t gi, uint32_t gj, void* st, dymu_stats* s) {
  (void)c; (void)F; (void)T; (void)nx; (void)ny; (void)ld; (void)gi; (void)gj; (void)st; (void)s; NODEV;
}
int dymu_solve_until_device(dymu_ctx* c, const double* F, double* T, uint32_t nx, uint32_t ny,
                            uint64_t ld, uint32_t gi, uint32_t gj, uint32_t si, uint32_t sj, void* st,
                            double* tc, dymu_stats* s) {
  (void)c; (void)F; (void)T; (void)nx; (void)ny; (void)ld; (void)gi; (void)gj; (void)si; (void)sj;
  (void)st; (void)tc; (void)s; NODEV;
}
int dymu_early_exit_mask(dymu_ctx* c, const double* F, double* T, uint32_t nx, uint32_t ny, uint64_t ld,
                         double tc, uint64_t* b, uint64_t cap, uint64_t* nb, void* st) {
  (void)c; (void)F; (void)T; (void)nx; (void)ny; (void)ld; (void)tc; (void)b; (void)cap; (void)nb; (void)st;
  NODEV;
}
int dymu_count_equal(dymu_ctx* c, const double* T, uint32_t nx, uint32_t ny, uint64_t ld, double v,
                     uint64_t* n, void* st) {
  (void)c; (void)T; (void)nx; (void)ny; (void)ld; (void)v; (void)n; (void)st; NODEV;
}
int dymu_find_equal(dymu_ctx* c, const double* T, uint32_t nx, uint32_t ny, uint64_t ld, double v,
                    uint64_t* idx, uint64_t cap, uint64_t* n, void* st) {
  (void)c; (void)T; (void)nx; (void)ny; (void)ld; (void)v; (void)idx; (void)cap; (void)n; (void)st;
  NODEV;
}
int dymu_region_stats(dymu_ctx* c, const double* F, const double* T, uint32_t nx, uint32_t ny,
                      uint64_t ld, uint32_t gi, uint32_t gj, double thr, double lo, double hi,
                      dymu_region* out, void* st) {
  (void)c; (void)F; (void)T; (void)nx; (void)ny; (void)ld; (void)gi; (void)gj; (void)thr;
  (void)lo; (void)hi; (void)out; (void)st; NODEV;
}
int dymu_scatter(dymu_ctx* c, double* T, uint32_t nx, uint64_t ld, const uint64_t* idx, const double* v,
                 uint64_t n, void* st) {
  (void)c; (void)T; (void)nx; (void)ld; (void)idx; (void)v; (void)n; (void)st; NODEV;
}
int dymu_update_window_device(dymu_ctx* c, const double* F, double* T, uint32_t nx, uint32_t ny,
                              uint64_t ld, uint32_t gi, uint32_t gj, uint32_t i0, uint32_t j0, uint32_t w,
                              uint32_t h, int dec, void* st, dymu_stats* s) {
  (void)c; (void)F; (void)T; (void)nx; (void)ny; (void)ld; (void)gi; (void)gj; (void)i0; (void)j0; (void)w;
  (void)h; (void)dec; (void)st; (void)s; NODEV;
}
