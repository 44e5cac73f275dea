// torch op registration for the gfx950 kernels (namespace `dcr`, loaded with
// torch.ops.load_library).  Only argument checking and stream plumbing lives here; every op
// launches hand-written HIP kernels from the *.hip files on the current HIP stream.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "kernels.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16")
#define CHECK_I32(t) TORCH_CHECK((t).scalar_type() == at::kInt, #t " must be int32")
#define CHECK_ALIGN16(t) \
  TORCH_CHECK((reinterpret_cast<uintptr_t>((t).data_ptr()) & 15) == 0, #t " must be 16-B aligned")

template <typename T>
T* ptr(const at::Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}
using bf16 = dcr::bf16;

// ------------------------------------------------------------------------------------------
// optimizer
// ------------------------------------------------------------------------------------------
void global_norm(const at::Tensor& g, at::Tensor& partials, at::Tensor& norm_out) {
  CHECK_DEV(g); CHECK_CONTIG(g); CHECK_F32(g); CHECK_ALIGN16(g);
  CHECK_F32(partials); CHECK_F32(norm_out);
  TORCH_CHECK(partials.numel() >= dcr::opt_num_partials(g.numel()), "partials too small");
  dcr::launch_global_norm(ptr<float>(g), g.numel(), ptr<float>(partials), ptr<float>(norm_out),
                          cur_stream());
}

void adam_clip(at::Tensor& p, const at::Tensor& g, at::Tensor& m, at::Tensor& v,
               const c10::optional<at::Tensor>& pbf, at::Tensor& partials, at::Tensor& norm_out,
               double lr_t, double b1, double b2, double eps, double clip) {
  for (const at::Tensor* t : {(const at::Tensor*)&p, &g, (const at::Tensor*)&m, (const at::Tensor*)&v}) {
    CHECK_DEV(*t); CHECK_CONTIG(*t); CHECK_F32(*t); CHECK_ALIGN16(*t);
    TORCH_CHECK(t->numel() == p.numel(), "adam buffers must have equal numel");
  }
  bf16* pb = nullptr;
  if (pbf.has_value() && pbf->defined()) {
    CHECK_BF16(*pbf); CHECK_CONTIG(*pbf); CHECK_ALIGN16(*pbf);
    TORCH_CHECK(pbf->numel() == p.numel(), "bf16 mirror numel mismatch");
    pb = ptr<bf16>(*pbf);
  }
  TORCH_CHECK(partials.numel() >= dcr::opt_num_partials(p.numel()), "partials too small");
  dcr::launch_adam_clip(ptr<float>(p), ptr<float>(g), ptr<float>(m), ptr<float>(v), pb,
                        p.numel(), ptr<float>(partials), ptr<float>(norm_out), (float)lr_t,
                        (float)b1, (float)b2, (float)eps, (float)clip, cur_stream());
}

}  // namespace

TORCH_LIBRARY(dcr, m) {
  m.def("opt_num_partials(int n) -> int", [](int64_t n) -> int64_t { return dcr::opt_num_partials(n); });
  m.def("global_norm(Tensor g, Tensor(a!) partials, Tensor(b!) norm_out) -> ()");
  m.def(
      "adam_clip(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor(d!)? pbf, "
      "Tensor(e!) partials, Tensor(f!) norm_out, float lr_t, float b1, float b2, float eps, "
      "float clip) -> ()");
}

TORCH_LIBRARY_IMPL(dcr, CUDA, m) {
  m.impl("global_norm", &global_norm);
  m.impl("adam_clip", &adam_clip);
}
