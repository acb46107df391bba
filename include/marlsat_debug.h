/* marlsat_debug.h — diagnostics exported by libmarlsat.so (not part of the
 * drop-in boundary; used by profiles/ablate.py to price the HBM write ceiling). */
#ifndef MARLSAT_DEBUG_H
#define MARLSAT_DEBUG_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* Fill `bytes` (multiple of 16) at dst with int32 `value` using 16 B stores on `grid` x 256 threads. */
int msat_debug_fill(void *dst, size_t bytes, int32_t value, int32_t nontemporal, int32_t grid, void *stream);
/* Same bytes, but block g writes one contiguous chunk [g*bytes/grid, (g+1)*bytes/grid). */
int msat_debug_fill_chunked(void *dst, size_t bytes, int32_t value, int32_t nontemporal, int32_t grid, void *stream);
#ifdef __cplusplus
}
#endif
#endif
