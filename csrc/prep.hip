// One launch for the per-step data movement around the persistent kernels.
//
// After every optimizer step the recurrent kernels need bf16 copies of the fp32 master weights in
// several layouts (W_h, W_hᵀ, W_x, W_xᵀ, the padded head matrices), and before each forward the
// initial state goes into slot 0 of the h/c sequence buffers and the hand-off counters are zeroed.
// Done with torch ops that was ~15 small kernels per step (~160 us of launches and gaps on
// MI355X, profiles/r1_v6_exclusive_fused_head.md).  Here the host builds a table of tasks over
// arbitrary row-strided 2-D views and ONE kernel executes it: each workgroup takes one 64x64 tile
// of one task.
//
//   COPY       dst[r, c]  = convert(src[r, c])           (fp32 -> bf16 or fp32 -> fp32)
//   TRANSPOSE  dst[c, r]  = convert(src[r, c])           64x64 tile staged through LDS
//   ZERO       dst[r, c]  = 0                            (4-byte elements; counters)
#include "common.h"
#include "kernels.h"

namespace dcr {

constexpr int kPrepTile = 64;

__global__ void __launch_bounds__(256) prep_kernel(PrepTable tab) {
  __shared__ float tile[kPrepTile][kPrepTile + 1];
  int bid = blockIdx.x, k = 0;
  while (k + 1 < tab.n && bid >= tab.t[k + 1].tile0) ++k;
  const PrepTask& T = tab.t[k];
  const int local = bid - T.tile0;
  const int tiles_c = (T.cols + kPrepTile - 1) / kPrepTile;
  const int r0 = (local / tiles_c) * kPrepTile, c0 = (local % tiles_c) * kPrepTile;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  if (T.mode == PREP_ZERO) {
    for (int r = r0 + ty; r < min(r0 + kPrepTile, T.rows); r += 4)
      if (c0 + tx < T.cols) reinterpret_cast<float*>(T.dst)[(size_t)r * T.dst_ld + c0 + tx] = 0.f;
    return;
  }
  auto put = [&](size_t idx, float v) {
    if (T.dst_bf16) reinterpret_cast<bf16*>(T.dst)[idx] = f2bf(v);
    else reinterpret_cast<float*>(T.dst)[idx] = v;
  };
  if (T.mode == PREP_COPY) {
    for (int r = r0 + ty; r < min(r0 + kPrepTile, T.rows); r += 4)
      if (c0 + tx < T.cols) put((size_t)r * T.dst_ld + c0 + tx, T.src[(size_t)r * T.src_ld + c0 + tx]);
    return;
  }
  // TRANSPOSE: coalesced read of rows r, coalesced write of dst rows c
  for (int r = ty; r < kPrepTile; r += 4)
    if (r0 + r < T.rows && c0 + tx < T.cols)
      tile[r][tx] = T.src[(size_t)(r0 + r) * T.src_ld + c0 + tx];
  __syncthreads();
  for (int c = ty; c < kPrepTile; c += 4)
    if (c0 + c < T.cols && r0 + tx < T.rows) put((size_t)(c0 + c) * T.dst_ld + r0 + tx, tile[tx][c]);
}

int prep_tiles(int rows, int cols) {
  return ((rows + kPrepTile - 1) / kPrepTile) * ((cols + kPrepTile - 1) / kPrepTile);
}

void launch_prep(PrepTable& tab, hipStream_t s) {
  int tiles = 0;
  for (int i = 0; i < tab.n; ++i) {
    tab.t[i].tile0 = tiles;
    tiles += prep_tiles(tab.t[i].rows, tab.t[i].cols);
  }
  if (tiles > 0) prep_kernel<<<tiles, 256, 0, s>>>(tab);
}

}  // namespace dcr
