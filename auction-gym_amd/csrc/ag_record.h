// ag_record.h -- indexing of the ABI 17 packed log record (include/auctiongym.h
// ag_batch_out.record), shared by the simulate kernels (writers) and the collect kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace ag {

// The log record {bid, est_ctr, true_ctr, best_ev} of (slot s, auction i).
// Record layouts (A/B; the ABI states kRecLayout):
//   0: [P][B][4] rows, two 16-B stores per lane (each wave store covers half of each line);
//   1: 64-auction tiles [P][T][4][64] (T = ceil(B / 64)), four 8-B stores, each 512 B contiguous;
//   2: 64-auction tiles of pairs [P][T][2][64][2], two 16-B stores, each 1 KB contiguous.
#ifndef AG_REC_LAYOUT
#define AG_REC_LAYOUT 2
#endif
constexpr int kRecLayout = AG_REC_LAYOUT;
__device__ __forceinline__ size_t rec_index(int layout, uint32_t s, uint32_t i, uint32_t B, int h) {
  // the double index of the record's half h (fields 2h, 2h + 1)
  if (layout == 0) return ((size_t)s * B + i) * 4 + 2 * h;
  const size_t tile = (size_t)s * ((B + 63) >> 6) + (i >> 6);
  if (layout == 1) return (tile * 4 + 2 * h) * 64 + (i & 63);
  return ((tile * 2 + h) * 64 + (i & 63)) * 2;
}
// the double index of field f (0 bid, 1 est_ctr, 2 true_ctr, 3 best_ev) of (s, i)
__device__ __forceinline__ size_t rec_field(int layout, uint32_t s, uint32_t i, uint32_t B, int f) {
  return rec_index(layout, s, i, B, f >> 1) + (layout == 1 ? (size_t)(f & 1) * 64 : (size_t)(f & 1));
}

}  // namespace ag
