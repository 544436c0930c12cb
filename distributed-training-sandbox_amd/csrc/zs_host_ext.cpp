// Host-side helper of the ZeRO-3 hooks (zero_amd/zero3.py): installs a module's gathered full
// tensors into its parameters, and puts the local shards back, in ONE call per module.
//
// The reference does this per parameter in Python (zero3.py:36-52: `param.data = full` after each
// all-gather, `param.data = shard` on release).  With one grouped gather per module the per-
// parameter Python left is a strided view of the gathered allocation plus a `.data` swap — about
// 2-4 us per parameter, 582 of each per iteration of the configs[4] set (291 tensors, gathered for
// forward and again for backward), a third of the hooked iteration's host time.  Here the loop runs
// in C++ and rewrites each parameter's storage / sizes / strides / offset in place — the metadata
// half of Tensor::set_data (`param.data = x`), no view tensors built.
//
// Built against the torch headers of this image (no HIP code): zero_amd/_hostext*.so.
#include <torch/extension.h>

#include <cstdint>
#include <vector>

namespace {

class ViewPlan {
 public:
  // params[i] takes hold.as_strided(sizes[i], strides[i], offsets[i]) on install() and shards[i]
  // on release()
  ViewPlan(std::vector<at::Tensor> params, std::vector<at::Tensor> shards,
           std::vector<std::vector<int64_t>> sizes, std::vector<std::vector<int64_t>> strides,
           std::vector<int64_t> offsets)
      : params_(std::move(params)), shards_(std::move(shards)), sizes_(std::move(sizes)),
        strides_(std::move(strides)), offsets_(std::move(offsets)) {
    const size_t n = params_.size();
    TORCH_CHECK(shards_.size() == n && sizes_.size() == n && strides_.size() == n &&
                    offsets_.size() == n,
                "ViewPlan: params, shards, sizes, strides and offsets differ in length");
    for (size_t i = 0; i < n; ++i) {
      TORCH_CHECK(sizes_[i].size() == strides_[i].size(), "ViewPlan: sizes / strides rank of ", i);
      TORCH_CHECK(offsets_[i] >= 0, "ViewPlan: negative offset of ", i);
      bool empty = false;
      int64_t last = offsets_[i];  // the highest element the view reaches
      for (size_t d = 0; d < sizes_[i].size(); ++d) {
        TORCH_CHECK(sizes_[i][d] >= 0 && strides_[i][d] >= 0, "ViewPlan: bad geometry of ", i);
        empty |= sizes_[i][d] == 0;
        if (sizes_[i][d] > 0) last += (sizes_[i][d] - 1) * strides_[i][d];
      }
      if (!empty) extent_ = std::max(extent_, last + 1);
    }
    for (size_t i = 0; i < n; ++i) {
      // the parameters' metadata is rewritten in place: same dtype and device everywhere, and
      // tensors that allow it (a Parameter does)
      TORCH_CHECK(params_[i].scalar_type() == params_[0].scalar_type() &&
                      params_[i].device() == params_[0].device() &&
                      shards_[i].scalar_type() == params_[0].scalar_type() &&
                      shards_[i].device() == params_[0].device(),
                  "ViewPlan: parameters and shards must share one dtype and device");
      TORCH_CHECK(params_[i].unsafeGetTensorImpl()->allow_tensor_metadata_change(),
                  "ViewPlan: parameter ", i, " does not allow metadata changes");
    }
    if (n) {
      dtype_ = params_[0].scalar_type();
      device_ = params_[0].device();
    }
  }

  // the views of `hold` (one per parameter), without touching the parameters
  std::vector<at::Tensor> views(const at::Tensor& hold) const {
    check_hold(hold);
    std::vector<at::Tensor> out;
    out.reserve(params_.size());
    for (size_t i = 0; i < params_.size(); ++i)
      out.push_back(hold.as_strided(sizes_[i], strides_[i], hold.storage_offset() + offsets_[i]));
    return out;
  }

  // every parameter's data becomes its view of `hold` — what `param.data = view` does (the
  // parameter's storage, sizes, strides and offset replaced; its version counter, autograd state
  // and dtype kept), without building the view tensors
  void install(const at::Tensor& hold) {
    check_hold(hold);
    const c10::Storage& st = hold.storage();
    const int64_t base = hold.storage_offset();
    for (size_t i = 0; i < params_.size(); ++i) {
      c10::TensorImpl* impl = params_[i].unsafeGetTensorImpl();
      impl->set_storage_keep_dtype(st);
      impl->set_sizes_and_strides(sizes_[i], strides_[i], base + offsets_[i]);
    }
  }

  // every parameter's data back to its local shard (`param.data = shard`)
  void release() {
    for (size_t i = 0; i < params_.size(); ++i) {
      c10::TensorImpl* impl = params_[i].unsafeGetTensorImpl();
      const at::Tensor& sh = shards_[i];
      impl->set_storage_keep_dtype(sh.storage());
      impl->set_sizes_and_strides(sh.sizes(), sh.strides(), sh.storage_offset());
    }
  }

  int64_t size() const { return static_cast<int64_t>(params_.size()); }
  int64_t extent() const { return extent_; }

 private:
  void check_hold(const at::Tensor& hold) const {
    TORCH_CHECK(hold.dim() == 1 && hold.is_contiguous(), "ViewPlan: hold must be 1-D contiguous");
    TORCH_CHECK(hold.numel() >= extent_, "ViewPlan: hold has ", hold.numel(),
                " elements, the views reach ", extent_);
    TORCH_CHECK(hold.scalar_type() == dtype_ && hold.device() == device_,
                "ViewPlan: hold's dtype / device differ from the parameters'");
  }

  std::vector<at::Tensor> params_, shards_;
  std::vector<std::vector<int64_t>> sizes_, strides_;
  std::vector<int64_t> offsets_;
  int64_t extent_ = 0;
  at::ScalarType dtype_ = at::kFloat;
  at::Device device_ = at::kCPU;
};

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "zero_amd host helper: per-module install / release of ZeRO-3 gathered parameters";
  pybind11::class_<ViewPlan>(m, "ViewPlan")
      .def(pybind11::init<std::vector<at::Tensor>, std::vector<at::Tensor>,
                          std::vector<std::vector<int64_t>>, std::vector<std::vector<int64_t>>,
                          std::vector<int64_t>>())
      .def("views", &ViewPlan::views)
      .def("install", &ViewPlan::install)
      .def("release", &ViewPlan::release)
      .def_property_readonly("size", &ViewPlan::size)
      .def_property_readonly("extent", &ViewPlan::extent);
}
