/* marlsat_probe.h — diagnostics exported by libmarlsat_probe.so (not part of the
 * drop-in boundary; used by profiles/ablate.py to price the HBM write ceiling). */
#ifndef MARLSAT_PROBE_H
#define MARLSAT_PROBE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* Fill `bytes` (multiple of 16) at dst with int32 `value` using 16 B stores on `grid` x 256 threads. */
int msat_probe_fill(void *dst, size_t bytes, int32_t value, int32_t nontemporal, int32_t grid, void *stream);
/* Same bytes, but block g writes one contiguous chunk [g*bytes/grid, (g+1)*bytes/grid). */
int msat_probe_fill_chunked(void *dst, size_t bytes, int32_t value, int32_t nontemporal, int32_t grid, void *stream);
/* Expand compact bit images into int32 obs [E][A][D] (D % 4 == 0): element (e, a, d) is
 * bit d of vimg[e] if bit d of mimg[inst[e]][a] is set, else -1 (two-phase env-step probe).
 * grid > 0: one lane per 16 B quad, grid-stride; grid < 0: -grid blocks, one wave per row. */
int msat_probe_obs_expand(void *dst, int32_t E, int32_t A, int32_t D, const int32_t *inst, const uint32_t *vimg,
                          const uint32_t *mimg, int32_t grid, void *stream);
/* One workgroup per env (grid-stride over E) writes its A rows of D16 x 16 B: env-major [E][A][D]
 * (amajor = 0) or agent-major [A][E][D] (amajor = 1); threads 256 or 512. */
int msat_probe_fill_rows(void *dst, int32_t E, int32_t A, int32_t D16, int32_t amajor, int32_t value, int32_t threads,
                         int32_t grid, void *stream);
/* Read M x K floats of D (leading dimension ld) as the data gradient's register-A column strips (mode 0),
 * as contiguous rows (1), or as strips with three workgroups per row block (2); out: one float per thread. */
int msat_probe_strip_read(const float *D, int32_t M, int32_t ld, int32_t K, int32_t mode, float *out, void *stream);
/* Texture-path probe: `grid` x 256 threads read an L2-resident window of `window` bytes, `iters` wave-
 * instructions of 1 KiB per wave, as plain loads (mode 0 lane-linear, 2 register-A pattern: 16 rows `stride`
 * bytes apart, 64 B each) or LDS-DMA pieces (1 lane-linear, 3 weight-piece pattern: 16 rows, 64 B each). */
int msat_probe_l2_read(const void *buf, int32_t window, int32_t mode, int32_t iters, int32_t grid, int32_t stride,
                       float *out, void *stream);
#ifdef __cplusplus
}
#endif
#endif
