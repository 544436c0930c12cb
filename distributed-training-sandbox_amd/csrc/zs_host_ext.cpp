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
// Round 6: GradCounter — the per-parameter post-accumulate-grad bookkeeping of the ZeRO-3 backward
// (zero3.py:56-77's hooks fire per parameter; the gradient reduce-scatter buckets and the
// per-module release count parameters) as C++ hooks on the parameters' AccumulateGrad: a
// parameter's completed gradient decrements its bucket's / module's count without entering
// Python, and Python is called once per completed bucket (or run of buckets) and once per
// released module instead of once per parameter and counter.
//
// Round 6, second pass: GatherFast / consume — a module gather's side-stream allocation, receive
// table and synced library call in one C++ call, and its consumption (the consumer's wait, the
// caching allocator's record of the consumer stream, the ViewPlan install) in another; device and
// stream handling through c10's device-generic guards, so still no HIP code here.
//
// Built against the torch headers of this image (no HIP code): zero_amd/_hostext*.so.
#include <Python.h>
#include <c10/core/StreamGuard.h>
#include <c10/core/impl/DeviceGuardImplInterface.h>
#include <torch/csrc/autograd/function_hook.h>
#include <torch/csrc/autograd/variable.h>
#include <torch/extension.h>

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

namespace {
namespace py = pybind11;

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

// Counts completed parameter gradients into slots.
//   ordered (gradient buckets): slot k's count drops by one per parameter; whenever the run of
//     completed slots from `next` grows, on_ready(new next) — the caller launches buckets
//     [old next, new next) in order; a parameter counted twice before reset() is an error
//     (the reference reduces each gradient once per step).
//   unordered (modules): a slot counts only while open (open(slot, n) at the module's backward
//     gather); when it reaches zero it closes and on_ready(slot) — the caller releases the module.
// on_first() (may be None) runs at the first count after reset(): the caller queues its
// end-of-backward callback from inside the backward.  Counting takes no GIL; the callbacks take it.
class GradCounter {
 public:
  GradCounter(std::vector<int64_t> sizes, int64_t n_params, bool ordered, py::object on_first,
              py::object on_ready, std::string twice_msg)
      : sizes_(std::move(sizes)), ordered_(ordered), on_first_(std::move(on_first)),
        on_ready_(std::move(on_ready)), twice_msg_(std::move(twice_msg)) {
    TORCH_CHECK(n_params >= 0, "GradCounter: n_params < 0");
    marked_.assign(static_cast<size_t>(n_params), 0);
    reset();
  }

  ~GradCounter() {
    if (Py_IsInitialized()) {
      py::gil_scoped_acquire g;
      on_first_ = py::object();
      on_ready_ = py::object();
    } else {  // interpreter gone: leak the two references rather than touch it
      on_first_.release();
      on_ready_.release();
    }
  }

  void reset() {
    std::lock_guard<std::mutex> lk(mu_);
    pending_ = ordered_ ? sizes_ : std::vector<int64_t>(sizes_.size(), 0);
    open_.assign(sizes_.size(), 0);
    std::fill(marked_.begin(), marked_.end(), 0);
    next_ = 0;
    first_ = true;
    counted_ = 0;
  }

  void open(int64_t slot, int64_t n) {
    std::lock_guard<std::mutex> lk(mu_);
    check_slot(slot);
    pending_[slot] = n;
    open_[slot] = n > 0;
  }

  void close_all() {
    std::lock_guard<std::mutex> lk(mu_);
    std::fill(open_.begin(), open_.end(), 0);
  }

  // one parameter's gradient is complete (param: its index for the twice check, or -1)
  void count(int64_t param, int64_t slot) {
    bool first = false;
    int64_t ready = -1;
    {
      std::lock_guard<std::mutex> lk(mu_);
      check_slot(slot);
      if (param >= 0 && static_cast<size_t>(param) < marked_.size()) {
        TORCH_CHECK(!marked_[param], twice_msg_, " (parameter ", param, ")");
        marked_[param] = 1;
      }
      ++counted_;
      first = first_;
      first_ = false;
      if (ordered_) {
        --pending_[slot];
        const int64_t old = next_;
        while (next_ < static_cast<int64_t>(pending_.size()) && pending_[next_] <= 0) ++next_;
        if (next_ != old) ready = next_;
      } else if (open_[slot] && --pending_[slot] == 0) {
        open_[slot] = 0;
        ready = slot;
      }
    }
    if (!first && ready < 0) return;
    py::gil_scoped_acquire g;
    if (first && !on_first_.is_none()) on_first_();
    if (ready >= 0 && !on_ready_.is_none()) on_ready_(ready);
  }

  int64_t next() const { return next_; }
  int64_t counted() const { return counted_; }
  std::vector<int64_t> pending() {
    std::lock_guard<std::mutex> lk(mu_);
    return pending_;
  }

 private:
  void check_slot(int64_t slot) const {
    TORCH_CHECK(slot >= 0 && static_cast<size_t>(slot) < sizes_.size(), "GradCounter: slot ", slot,
                " out of range [0, ", sizes_.size(), ")");
  }

  std::mutex mu_;
  std::vector<int64_t> sizes_, pending_;
  std::vector<uint8_t> open_, marked_;
  bool ordered_;
  int64_t next_ = 0, counted_ = 0;
  bool first_ = true;
  py::object on_first_, on_ready_;
  std::string twice_msg_;
};

// The parameter's post-accumulate-grad hook slot holds ONE object (torch keeps its Python hooks
// dict in it, torch/csrc/autograd/variable.h): this one runs whatever it replaced (the Python
// hooks) first, then counts into its targets — a counter's callback may launch the gradient's
// reduce-scatter and drop p.grad, so every Python hook, registered before the counter or after,
// still sees the gradient backward produced.  attach() first makes sure the Python dict exists,
// so a later Python registration adds to it instead of replacing the slot.
struct CountingHook : torch::autograd::PostAccumulateGradHook {
  std::vector<std::tuple<std::shared_ptr<GradCounter>, int64_t, int64_t>> targets;
  std::unique_ptr<torch::autograd::PostAccumulateGradHook> prev;

  void operator()(const torch::autograd::Variable& t) override {
    if (prev) (*prev)(t);
    const auto tg = targets;  // (a callback may detach a target)
    for (const auto& [c, param, slot] : tg) c->count(param, slot);
  }
};

void attach(const at::Tensor& param, const std::shared_ptr<GradCounter>& counter, int64_t index,
            int64_t slot) {
  TORCH_CHECK(param.requires_grad() && param.is_leaf(),
              "attach: the tensor must be a leaf that requires grad");
  auto& hook = torch::autograd::impl::post_acc_grad_hooks(param);
  auto* ch = dynamic_cast<CountingHook*>(hook.get());
  if (ch == nullptr) {
    auto h = std::make_unique<CountingHook>();
    h->prev = std::move(hook);
    ch = h.get();
    torch::autograd::impl::set_post_acc_grad_hooks(param, std::move(h));
  }
  ch->targets.emplace_back(counter, index, slot);
}

// drop every target of `counter` from the parameter's hook (the hook object itself stays: it may
// be running — a callback detaching from inside the backward — and passes through to `prev`)
void detach(const at::Tensor& param, const std::shared_ptr<GradCounter>& counter) {
  auto& hook = torch::autograd::impl::post_acc_grad_hooks(param);
  auto* ch = dynamic_cast<CountingHook*>(hook.get());
  if (ch == nullptr) return;
  auto& tg = ch->targets;
  tg.erase(std::remove_if(tg.begin(), tg.end(),
                          [&](const auto& t) { return std::get<0>(t) == counter; }),
           tg.end());
}

int64_t attached(const at::Tensor& param) {
  auto& hook = torch::autograd::impl::post_acc_grad_hooks(param);
  auto* ch = dynamic_cast<CountingHook*>(hook.get());
  return ch == nullptr ? -1 : static_cast<int64_t>(ch->targets.size());
}

// One module's side-stream gather, issued and consumed in one call each (round 6, second pass).
// What _GatherRuntime's Python did per gather — allocate the module's full tensors on the side
// stream, point the table's receive addresses into the allocation, call the library's synced group
// (ready wait, the RCCL group of all-gathers, the done record) — and per consumption — the
// consumer's wait, the allocator's record of the consumer stream, the ViewPlan install.  The
// library entry points come in as addresses (zs_all_gather_group_synced / zs_sync_wait, include/
// zero_amd.h): this helper is not linked against libzero_amd.so.
using SyncedGroupFn = int (*)(void* comm, int64_t n, const uint64_t* send, const uint64_t* recv,
                              const int64_t* count, int dtype, uintptr_t after, void* ready,
                              uintptr_t stream, void* done);
using SyncWaitFn = int (*)(void* sync, uintptr_t stream);

class GatherFast {
 public:
  // fn: the synced group's address; comm: the communicator handle (0 with n_coll = 0: the
  // ordering alone, no collective — the simulated-rank benches); send / count: the module's
  // chunk-arena slots and element counts; offs: each full tensor's byte offset in the allocation
  GatherFast(uintptr_t fn, uintptr_t comm, bool collective, std::vector<uint64_t> send,
             std::vector<int64_t> count, std::vector<uint64_t> offs, int64_t total, int zdtype,
             at::ScalarType dtype, int64_t device_index)
      : fn_(reinterpret_cast<SyncedGroupFn>(fn)), comm_(reinterpret_cast<void*>(comm)),
        collective_(collective), send_(std::move(send)), count_(std::move(count)),
        offs_(std::move(offs)), total_(total), zdtype_(zdtype), dtype_(dtype),
        device_(c10::DeviceType::CUDA, static_cast<c10::DeviceIndex>(device_index)) {
    TORCH_CHECK(fn_ != nullptr, "GatherFast: NULL group function");
    TORCH_CHECK(send_.size() == count_.size() && send_.size() == offs_.size(),
                "GatherFast: send, count and offs differ in length");
    TORCH_CHECK(total_ > 0, "GatherFast: total must be > 0");
    recv_.assign(send_.size(), 0);
  }

  // allocate on the side stream (side_id: its torch stream id), fill the receive table, enqueue
  // the synced group; returns (status, allocation)
  std::tuple<int, at::Tensor> launch(uintptr_t after, uintptr_t ready, int64_t side_id,
                                     uintptr_t side_h, uintptr_t done) {
    at::Tensor hold;
    {
      c10::StreamGuard g(c10::Stream::unpack3(side_id, device_.index(), c10::DeviceType::CUDA));
      hold = at::empty({total_}, at::TensorOptions().dtype(dtype_).device(device_));
    }
    const uint64_t base = reinterpret_cast<uint64_t>(hold.data_ptr());
    for (size_t i = 0; i < recv_.size(); ++i) recv_[i] = base + offs_[i];
    const int64_t n = collective_ ? static_cast<int64_t>(send_.size()) : 0;
    const int rc = fn_(comm_, n, n ? send_.data() : nullptr, n ? recv_.data() : nullptr,
                       n ? count_.data() : nullptr, zdtype_, after, reinterpret_cast<void*>(ready),
                       side_h, reinterpret_cast<void*>(done));
    return {rc, hold};
  }

  int64_t size() const { return static_cast<int64_t>(send_.size()); }

 private:
  SyncedGroupFn fn_;
  void* comm_;
  bool collective_;
  std::vector<uint64_t> send_, recv_;
  std::vector<int64_t> count_;
  std::vector<uint64_t> offs_;
  int64_t total_;
  int zdtype_;
  at::ScalarType dtype_;
  c10::Device device_;
};

// One gradient bucket's reduce-scatter issued in one call (update mode's _GradReducer._launch):
// every parameter's gradient must be there, dense, of the bucket's dtype and exactly ws chunks
// long (zero-copy: the gradient itself is the send buffer) — otherwise launch() returns -1 and
// touches nothing, and the caller takes its general path.  Then the send table, the library's
// synced group (ready wait, the RCCL group of reduce-scatters, the done record), the allocator's
// record of the collective stream on each gradient (`record`: it is read there after the
// gradient is dropped) and `p.grad = None` for each.
class ReduceFast {
 public:
  ReduceFast(uintptr_t fn, uintptr_t comm, bool collective, std::vector<at::Tensor> params,
             std::vector<uint64_t> recv, std::vector<int64_t> count, int zdtype,
             at::ScalarType dtype, int64_t ws)
      : fn_(reinterpret_cast<SyncedGroupFn>(fn)), comm_(reinterpret_cast<void*>(comm)),
        collective_(collective), params_(std::move(params)), recv_(std::move(recv)),
        count_(std::move(count)), zdtype_(zdtype), dtype_(dtype), ws_(ws) {
    TORCH_CHECK(fn_ != nullptr, "ReduceFast: NULL group function");
    TORCH_CHECK(params_.size() == recv_.size() && params_.size() == count_.size(),
                "ReduceFast: params, recv and count differ in length");
    send_.assign(params_.size(), 0);
    grads_.resize(params_.size());
  }

  int launch(uintptr_t after, uintptr_t ready, int64_t stream_id, int64_t device_index,
             uintptr_t stream_h, uintptr_t done, bool record) {
    for (size_t i = 0; i < params_.size(); ++i) {
      const at::Tensor& g = params_[i].grad();
      if (!g.defined() || g.scalar_type() != dtype_ || !g.is_contiguous() ||
          g.numel() != ws_ * count_[i])
        return -1;
      grads_[i] = g;
      send_[i] = reinterpret_cast<uint64_t>(g.data_ptr());
    }
    const int64_t n = collective_ ? static_cast<int64_t>(params_.size()) : 0;
    const int rc = fn_(comm_, n, n ? send_.data() : nullptr, n ? recv_.data() : nullptr,
                       n ? count_.data() : nullptr, zdtype_, after, reinterpret_cast<void*>(ready),
                       stream_h, reinterpret_cast<void*>(done));
    if (rc == 0) {
      const c10::Stream st = c10::Stream::unpack3(
          stream_id, static_cast<c10::DeviceIndex>(device_index), c10::DeviceType::CUDA);
      for (size_t i = 0; i < params_.size(); ++i) {
        if (record) grads_[i].record_stream(st);
        params_[i].mutable_grad().reset();
      }
    }
    for (auto& g : grads_) g.reset();
    return rc;
  }

 private:
  SyncedGroupFn fn_;
  void* comm_;
  bool collective_;
  std::vector<at::Tensor> params_, grads_;
  std::vector<uint64_t> recv_, send_;
  std::vector<int64_t> count_;
  int zdtype_;
  at::ScalarType dtype_;
  int64_t ws_;
};

// The consumer's side of a gather: wait on `wait_sync` (0: none) on the current stream `cur_h`,
// record the current stream's use of `hold` with the caching allocator (`record`), install the
// module's parameters from it.  Returns the wait's status.
int consume(uintptr_t wait_fn, uintptr_t wait_sync, uintptr_t cur_h, const at::Tensor& hold,
            ViewPlan& vp, bool record) {
  if (wait_sync) {
    const int rc = reinterpret_cast<SyncWaitFn>(wait_fn)(reinterpret_cast<void*>(wait_sync), cur_h);
    if (rc) return rc;
  }
  if (record) {
    const auto* impl = c10::impl::getDeviceGuardImpl(hold.device().type());
    hold.record_stream(impl->getStream(hold.device()));
  }
  vp.install(hold);
  return 0;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "zero_amd host helper: per-module install / release of ZeRO-3 gathered parameters, "
            "and the per-parameter gradient counting of the ZeRO-3 backward";
  pybind11::class_<ViewPlan>(m, "ViewPlan")
      .def(pybind11::init<std::vector<at::Tensor>, std::vector<at::Tensor>,
                          std::vector<std::vector<int64_t>>, std::vector<std::vector<int64_t>>,
                          std::vector<int64_t>>())
      .def("views", &ViewPlan::views)
      .def("install", &ViewPlan::install)
      .def("release", &ViewPlan::release)
      .def_property_readonly("size", &ViewPlan::size)
      .def_property_readonly("extent", &ViewPlan::extent);
  pybind11::class_<GradCounter, std::shared_ptr<GradCounter>>(m, "GradCounter")
      .def(pybind11::init<std::vector<int64_t>, int64_t, bool, py::object, py::object, std::string>(),
           py::arg("sizes"), py::arg("n_params"), py::arg("ordered"), py::arg("on_first"),
           py::arg("on_ready"), py::arg("twice_msg") = "gradient accumulated twice before reset")
      .def("reset", &GradCounter::reset)
      .def("open", &GradCounter::open)
      .def("close_all", &GradCounter::close_all)
      .def("count", &GradCounter::count, py::call_guard<py::gil_scoped_release>())
      .def("pending", &GradCounter::pending)
      .def_property_readonly("next", &GradCounter::next)
      .def_property_readonly("counted", &GradCounter::counted);
  pybind11::class_<GatherFast>(m, "GatherFast")
      .def(pybind11::init<uintptr_t, uintptr_t, bool, std::vector<uint64_t>, std::vector<int64_t>,
                          std::vector<uint64_t>, int64_t, int, at::ScalarType, int64_t>())
      .def("launch", &GatherFast::launch)
      .def_property_readonly("size", &GatherFast::size);
  m.def("consume", &consume, "the consumer's wait, the allocator's stream record, the install");
  pybind11::class_<ReduceFast>(m, "ReduceFast")
      .def(pybind11::init<uintptr_t, uintptr_t, bool, std::vector<at::Tensor>, std::vector<uint64_t>,
                          std::vector<int64_t>, int, at::ScalarType, int64_t>())
      .def("launch", &ReduceFast::launch);
  m.def("attach", &attach, "count `param`'s completed gradients into counter slot `slot`");
  m.def("detach", &detach, "drop every target of `counter` from `param`'s hook");
  m.def("attached", &attached, "targets on `param`'s counting hook (-1: none installed)");
}
