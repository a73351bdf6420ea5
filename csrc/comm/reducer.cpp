// Native DDP gradient reducer (``mipipe._C.Reducer``) — SURVEY §5.8 design item 1.
//
// Replaces the C++ Reducer behind the reference's ``DistributedDataParallel(model,
// device_ids=[args.gpu])`` (/root/reference/task.py:189; hot loop :309-311), built around
// mipipe's flat gradient buffer instead of per-bucket staging copies:
//
//  * buckets are contiguous [start, end) slices of the ONE flat fp32 gradient buffer
//    (mipipe.optim.flat), laid out in gradient-ready order, so RCCL reduces them in place;
//  * readiness is counted here, natively: a post hook on every parameter's AccumulateGrad node
//    (no Python frame per parameter; the node is looked up under the forward's stream, so
//    eager steps and hipGraph captures on a side stream both keep their stream) plus
//    ``mark_ready(slot)`` for the HIP kernels that write a weight gradient straight into the
//    flat buffer; a slot reported twice counts once;
//  * buckets launch strictly in index order (every rank issues the same collective sequence)
//    through the c10d ProcessGroup resolved by name — on ROCm the "nccl" backend is RCCL, its
//    work runs on the PG's own (high-priority, see parallel/dist_utils.py) HIP stream, ordered
//    after the gradient kernels on the caller's stream by the PG's event dependency;
//  * the end-of-backward engine callback launches what is left (unused parameters still take
//    part in the average) and makes the compute stream wait on every bucket — stream semantics,
//    the host never blocks on RCCL;
//  * averaging is RCCL's ncclAvg (ReduceOp.AVG); with the bf16 wire format one HIP pass packs
//    the bucket pre-scaled by 1/world (``grad_pack_bf16``), the reduction is a SUM of halves as
//    many bytes, and one pass widens it back (``grad_unpack_bf16``).  On gloo (CPU tests) the
//    same steps run as ATen ops.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/function_hook.h>
#include <torch/csrc/autograd/variable.h>
#include <torch/csrc/distributed/c10d/GroupRegistry.hpp>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "kernels/launchers.hpp"

namespace py = pybind11;

namespace mipipe_comm {

class Reducer : public std::enable_shared_from_this<Reducer> {
 public:
  Reducer(const std::string& group_name, at::Tensor flat_grad,
          std::vector<std::pair<int64_t, int64_t>> buckets, std::vector<int64_t> slot_bucket,
          int64_t world, bool avg, bool wire_bf16)
      : pg_(c10d::resolve_process_group(group_name)),
        flat_(std::move(flat_grad)),
        bounds_(std::move(buckets)),
        slot_bucket_(std::move(slot_bucket)),
        world_(world),
        avg_(avg),
        wire_bf16_(wire_bf16) {
    TORCH_CHECK(flat_.scalar_type() == at::kFloat && flat_.dim() == 1 && flat_.is_contiguous(),
                "Reducer: the flat gradient must be a contiguous 1-D float32 tensor");
    TORCH_CHECK(world_ >= 1, "Reducer: world size must be >= 1");
    const int64_t n = flat_.numel();
    members_.assign(bounds_.size(), 0);
    for (size_t b = 0; b < bounds_.size(); ++b) {
      const auto& r = bounds_[b];
      TORCH_CHECK(r.first >= 0 && r.first < r.second && r.second <= n,
                  "Reducer: bucket ", b, " [", r.first, ", ", r.second, ") outside the buffer");
      TORCH_CHECK(r.first % 8 == 0 && r.second % 8 == 0,
                  "Reducer: bucket bounds must be multiples of 8 elements");
      if (b > 0) TORCH_CHECK(r.first >= bounds_[b - 1].second, "Reducer: buckets must be ordered");
    }
    for (int64_t b : slot_bucket_) {
      TORCH_CHECK(b >= 0 && b < (int64_t)bounds_.size(), "Reducer: slot maps to bucket ", b);
      members_[b]++;
    }
    if (wire_bf16_) wire_ = at::empty({n}, flat_.options().dtype(at::kBFloat16));
    works_.resize(bounds_.size());
    pending_ = members_;
    reported_.assign(slot_bucket_.size(), 0);
  }

  ~Reducer() { remove_hooks(); }

  // Parameters whose AccumulateGrad nodes get the readiness post hook (slot i = params[i]).
  // The nodes are NOT created here: a node remembers the stream current at its creation and
  // the engine runs it there, so a node made at construction (default stream) would pin every
  // later backward — and a hipGraph capture on a side stream — to that stream ("unjoined
  // work").  prepare() creates / looks them up under the forward's stream instead.
  void register_hooks(const std::vector<at::Tensor>& params) {
    TORCH_CHECK(params.size() == slot_bucket_.size(), "Reducer: ", params.size(),
                " params for ", slot_bucket_.size(), " slots");
    std::lock_guard<std::mutex> g(mu_);
    params_ = params;
    hooked_.assign(params.size(), {});
    armed_.clear();
  }

  void remove_hooks() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& h : hooked_)
      if (auto n = h.first.lock()) n->del_post_hook(h.second);
    hooked_.clear();
    armed_.clear();
  }

  // Called at every grad-enabled forward, before the module runs: the next backward's
  // readiness starts from zero, and every parameter's current AccumulateGrad node carries the
  // hook.  The nodes are held until the end of that backward (a leaf keeps only a weak
  // reference: without this the node could die before the forward uses it).
  void prepare(bool enabled) {
    std::lock_guard<std::mutex> g(mu_);
    enabled_ = enabled;
    pending_ = members_;
    std::fill(reported_.begin(), reported_.end(), 0);
    for (auto& w : works_) w.reset();
    next_ = 0;
    callback_queued_ = false;
    armed_.clear();
    if (!enabled) return;
    std::weak_ptr<Reducer> self = shared_from_this();
    for (size_t i = 0; i < params_.size(); ++i) {
      auto acc = torch::autograd::impl::grad_accumulator(params_[i]);
      TORCH_CHECK(acc, "Reducer: parameter ", i, " has no grad accumulator (requires_grad?)");
      if (hooked_[i].first.lock() != acc) {
        auto key = acc->add_post_hook(std::make_unique<ReadyHook>(self, (int64_t)i));
        hooked_[i] = {acc, key};
      }
      armed_.push_back(std::move(acc));
    }
  }

  void mark_ready(int64_t slot) {
    std::lock_guard<std::mutex> g(mu_);
    if (!enabled_) return;
    TORCH_CHECK(slot >= 0 && slot < (int64_t)reported_.size(), "Reducer: bad slot ", slot);
    if (reported_[slot]) return;
    reported_[slot] = 1;
    if (!callback_queued_) {
      callback_queued_ = true;
      std::weak_ptr<Reducer> self = shared_from_this();
      torch::autograd::Engine::get_default_engine().queue_callback([self]() {
        if (auto r = self.lock()) r->finalize();
      });
    }
    --pending_[slot_bucket_[slot]];
    while (next_ < (int64_t)bounds_.size() && pending_[next_] <= 0) launch(next_++);
  }

  // End of backward: launch what is left, then make the caller's stream wait on every bucket.
  void finalize() {
    std::lock_guard<std::mutex> g(mu_);
    if (!enabled_) return;
    while (next_ < (int64_t)bounds_.size()) launch(next_++);
    for (size_t b = 0; b < works_.size(); ++b) {
      if (!works_[b]) continue;
      works_[b]->wait();
      works_[b].reset();
      at::Tensor slice = bucket_view(flat_, b);
      if (wire_bf16_) {
        at::Tensor w = bucket_view(wire_, b);
        if (slice.is_cuda())
          mipipe::grad_unpack_bf16(w.data_ptr(), slice.data_ptr<float>(), slice.numel(), stream());
        else
          slice.copy_(w);
      } else if (!avg_) {
        slice.div_((double)world_);
      }
    }
    ++steps_;
    callback_queued_ = false;
    armed_.clear();
  }

  int64_t launched() const { return launched_; }
  int64_t steps() const { return steps_; }
  int64_t num_buckets() const { return (int64_t)bounds_.size(); }
  bool wire_bf16() const { return wire_bf16_; }

 private:
  struct ReadyHook : torch::autograd::FunctionPostHook {
    ReadyHook(std::weak_ptr<Reducer> r, int64_t s) : r_(std::move(r)), slot_(s) {}
    torch::autograd::variable_list operator()(const torch::autograd::variable_list& outputs,
                                              const torch::autograd::variable_list&) override {
      if (auto r = r_.lock()) r->mark_ready(slot_);
      return outputs;
    }
    std::weak_ptr<Reducer> r_;
    int64_t slot_;
  };

  static hipStream_t stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

  at::Tensor bucket_view(const at::Tensor& buf, size_t b) const {
    return buf.narrow(0, bounds_[b].first, bounds_[b].second - bounds_[b].first);
  }

  void launch(int64_t b) {
    at::Tensor t = bucket_view(flat_, b);
    c10d::AllreduceOptions o;
    if (wire_bf16_) {
      at::Tensor w = bucket_view(wire_, b);
      const float scale = 1.0f / (float)world_;
      if (t.is_cuda())
        mipipe::grad_pack_bf16(t.data_ptr<float>(), w.data_ptr(), t.numel(), scale, stream());
      else
        w.copy_(t * scale);
      t = w;
      o.reduceOp = c10d::ReduceOp(c10d::ReduceOp::SUM);
    } else {
      o.reduceOp = c10d::ReduceOp(avg_ ? c10d::ReduceOp::AVG : c10d::ReduceOp::SUM);
    }
    std::vector<at::Tensor> ts{t};
    works_[b] = pg_->allreduce(ts, o);
    ++launched_;
  }

  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  at::Tensor flat_, wire_;
  std::vector<std::pair<int64_t, int64_t>> bounds_;
  std::vector<int64_t> slot_bucket_;
  std::vector<int64_t> members_, pending_;
  std::vector<char> reported_;
  std::vector<c10::intrusive_ptr<c10d::Work>> works_;
  std::vector<at::Tensor> params_;
  std::vector<std::pair<std::weak_ptr<torch::autograd::Node>, uintptr_t>> hooked_;
  std::vector<std::shared_ptr<torch::autograd::Node>> armed_;
  int64_t world_;
  bool avg_, wire_bf16_;
  bool enabled_ = true;
  bool callback_queued_ = false;
  int64_t next_ = 0;
  int64_t launched_ = 0;
  int64_t steps_ = 0;
  std::mutex mu_;
};

// Standalone wire-format passes (tests, and the Python fallback reducer on the GPU).
void grad_pack_bf16(const at::Tensor& g, at::Tensor& wire, double scale) {
  TORCH_CHECK(g.is_cuda() && wire.is_cuda(), "grad_pack_bf16: GPU tensors");
  TORCH_CHECK(g.scalar_type() == at::kFloat && wire.scalar_type() == at::kBFloat16,
              "grad_pack_bf16: float32 -> bfloat16");
  TORCH_CHECK(g.is_contiguous() && wire.is_contiguous() && g.numel() == wire.numel(),
              "grad_pack_bf16: contiguous tensors of equal size");
  TORCH_CHECK(g.numel() % 8 == 0 && (uintptr_t)g.data_ptr() % 16 == 0 &&
                  (uintptr_t)wire.data_ptr() % 16 == 0,
              "grad_pack_bf16: numel % 8 == 0 and 16-byte aligned storage");
  mipipe::grad_pack_bf16(g.data_ptr<float>(), wire.data_ptr(), g.numel(), (float)scale,
                         at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
}

void grad_unpack_bf16(const at::Tensor& wire, at::Tensor& g) {
  TORCH_CHECK(g.is_cuda() && wire.is_cuda(), "grad_unpack_bf16: GPU tensors");
  TORCH_CHECK(g.scalar_type() == at::kFloat && wire.scalar_type() == at::kBFloat16,
              "grad_unpack_bf16: bfloat16 -> float32");
  TORCH_CHECK(g.is_contiguous() && wire.is_contiguous() && g.numel() == wire.numel(),
              "grad_unpack_bf16: contiguous tensors of equal size");
  TORCH_CHECK(g.numel() % 8 == 0 && (uintptr_t)g.data_ptr() % 16 == 0 &&
                  (uintptr_t)wire.data_ptr() % 16 == 0,
              "grad_unpack_bf16: numel % 8 == 0 and 16-byte aligned storage");
  mipipe::grad_unpack_bf16(wire.data_ptr(), g.data_ptr<float>(), g.numel(),
                           at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
}

void init_comm(py::module& m) {
  py::class_<Reducer, std::shared_ptr<Reducer>>(m, "Reducer")
      .def(py::init<const std::string&, at::Tensor, std::vector<std::pair<int64_t, int64_t>>,
                    std::vector<int64_t>, int64_t, bool, bool>(),
           py::arg("group_name"), py::arg("flat_grad"), py::arg("buckets"),
           py::arg("slot_bucket"), py::arg("world"), py::arg("avg"), py::arg("wire_bf16"))
      .def("register_hooks", &Reducer::register_hooks)
      .def("remove_hooks", &Reducer::remove_hooks)
      .def("prepare", &Reducer::prepare, py::arg("enabled") = true)
      .def("mark_ready", &Reducer::mark_ready, py::call_guard<py::gil_scoped_release>())
      .def("finalize", &Reducer::finalize, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("launched", &Reducer::launched)
      .def_property_readonly("steps", &Reducer::steps)
      .def_property_readonly("num_buckets", &Reducer::num_buckets)
      .def_property_readonly("wire_bf16", &Reducer::wire_bf16);
  m.def("grad_pack_bf16", &grad_pack_bf16, py::arg("g"), py::arg("wire"), py::arg("scale"));
  m.def("grad_unpack_bf16", &grad_unpack_bf16, py::arg("wire"), py::arg("g"));
}

}  // namespace mipipe_comm
