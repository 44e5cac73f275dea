// Host-side launcher declarations for the gfx950 kernels.  Implemented in the *.hip files,
// bound to torch in ops.cpp.  All launchers are asynchronous on `stream`, allocate nothing and
// never synchronise (hipGraph-capturable, cdna_hip_programming.md Guideline 9).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dcr {
typedef __bf16 bf16;

// ---- optim.hip -------------------------------------------------------------------------
int opt_num_partials(int64_t n);
void launch_global_norm(const float* g, int64_t n, float* partials, float* norm_out,
                        hipStream_t stream);
void launch_adam_clip(float* p, const float* g, float* m, float* v, bf16* pbf, int64_t n,
                      float* partials, float* norm_out, float lr_t, float b1, float b2, float eps,
                      float clip, hipStream_t stream);

}  // namespace dcr
