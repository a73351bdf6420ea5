// Host side of the one-shot collectives (``mipipe._C.OneShot``; kernel: csrc/kernels/oneshot.hip).
//
// A workspace per rank = 4 KB of flags / counters + two data slots of `cap` bytes, allocated with
// hipMalloc and exported with hipIpcGetMemHandle; every rank maps every peer's workspace
// (hipIpcOpenMemHandle) after the handles were exchanged over the process group
// (mipipe/parallel/oneshot.py).  All ranks must be on one node (xGMI peers) and issue the same
// sequence of calls with the same sizes; a call never blocks the host (stream-ordered kernel).
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime_api.h>

#include <cstring>
#include <string>
#include <vector>

#include "kernels/launchers.hpp"

namespace py = pybind11;

namespace mipipe_comm {

#define OS_CHECK(expr)                                                                  \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    TORCH_CHECK(e_ == hipSuccess, "OneShot: ", #expr, " failed: ", hipGetErrorString(e_)); \
  } while (0)

class OneShot {
 public:
  OneShot(int rank, int world, int64_t cap_bytes, int device, double timeout_s)
      : rank_(rank), world_(world), cap_((cap_bytes + 4095) / 4096 * 4096), device_(device),
        timeout_s_(timeout_s) {
    TORCH_CHECK(world >= 1 && world <= 8, "OneShot: 1..8 ranks (one xGMI node), got ", world);
    TORCH_CHECK(rank >= 0 && rank < world, "OneShot: bad rank ", rank);
    TORCH_CHECK(cap_bytes > 0 && cap_bytes <= (64ll << 20), "OneShot: cap must be in (0, 64 MiB]");
    TORCH_CHECK(timeout_s > 0.0 && timeout_s < 1e5, "OneShot: timeout_s must be in (0, 1e5)");
    nblocks_ = mipipe::oneshot_blocks(cap_);
    OS_CHECK(hipSetDevice(device_));
    OS_CHECK(hipMalloc(&own_, mipipe::kOneShotHeaderBytes + 2 * cap_));
    OS_CHECK(hipMemset(own_, 0, mipipe::kOneShotHeaderBytes));  // flags, error words, counters
    OS_CHECK(hipHostMalloc(reinterpret_cast<void**>(&err_host_), 2 * sizeof(unsigned int),
                           hipHostMallocDefault));
    err_host_[0] = err_host_[1] = 0;
    OS_CHECK(hipEventCreateWithFlags(&err_ev_, hipEventDisableTiming));
    OS_CHECK(hipDeviceSynchronize());
    bases_.assign(world_, nullptr);
    bases_[rank_] = own_;
  }

  ~OneShot() {
    hipSetDevice(device_);
    for (int r = 0; r < world_; ++r)
      if (r != rank_ && bases_[r] != nullptr) hipIpcCloseMemHandle(bases_[r]);
    if (err_ev_ != nullptr) hipEventDestroy(err_ev_);
    if (err_host_ != nullptr) hipHostFree(err_host_);
    if (own_ != nullptr) hipFree(own_);
  }

  py::bytes handle() const {
    hipIpcMemHandle_t h;
    OS_CHECK(hipIpcGetMemHandle(&h, own_));
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }

  void open(const std::vector<std::string>& handles) {
    TORCH_CHECK((int)handles.size() == world_, "OneShot: ", handles.size(), " handles for ",
                world_, " ranks");
    OS_CHECK(hipSetDevice(device_));
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      TORCH_CHECK(handles[r].size() == sizeof(hipIpcMemHandle_t), "OneShot: bad handle size");
      hipIpcMemHandle_t h;
      std::memcpy(&h, handles[r].data(), sizeof(h));
      void* p = nullptr;
      OS_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      bases_[r] = static_cast<char*>(p);
    }
    opened_ = true;
  }

  // In place: t = sum over ranks (times 1/world when avg).  fp32, contiguous, 16-B multiple.
  void all_reduce(at::Tensor t, bool avg) {
    check(t, true);
    mipipe::oneshot_launch(bases_.data(), rank_, world_, t.data_ptr(), t.data_ptr(),
                           t.numel() * 4, true, 0, avg ? 1.0f / world_ : 1.0f, cap_, nblocks_,
                           timeout_s_, stream());
  }

  // In place: t = rank src's t (any dtype; byte size a multiple of 16).
  void broadcast(at::Tensor t, int src) {
    check(t, false);
    TORCH_CHECK(src >= 0 && src < world_, "OneShot: bad src ", src);
    mipipe::oneshot_launch(bases_.data(), rank_, world_, t.data_ptr(), t.data_ptr(),
                           t.numel() * t.element_size(), false, src, 1.0f, cap_, nblocks_,
                           timeout_s_, stream());
  }

  // Host read of the error words (synchronises the device): {1 + peer, epoch}; peer word 0 =
  // no wait ever gave up.
  std::pair<int, int64_t> error_info() const {
    unsigned int v[2] = {0, 0};
    OS_CHECK(hipDeviceSynchronize());
    OS_CHECK(hipMemcpy(v, own_ + mipipe::kOneShotErrOffset, 8, hipMemcpyDeviceToHost));
    return {(int)v[0], (int64_t)v[1]};
  }
  int error() const { return error_info().first; }

  // Asynchronous error check without a host sync: request_error() enqueues a copy of the error
  // words into pinned host memory on the current stream; poll_error() returns the words of the
  // last request once that copy has completed, else {-1, -1} (not known yet).
  void request_error() {
    OS_CHECK(hipMemcpyAsync(err_host_, own_ + mipipe::kOneShotErrOffset, 8,
                            hipMemcpyDeviceToHost, stream()));
    OS_CHECK(hipEventRecord(err_ev_, stream()));
    requested_ = true;
  }
  std::pair<int, int64_t> poll_error() const {
    if (!requested_) return {-1, -1};
    const hipError_t q = hipEventQuery(err_ev_);
    if (q == hipErrorNotReady) return {-1, -1};
    OS_CHECK(q);
    return {(int)err_host_[0], (int64_t)err_host_[1]};
  }

  int64_t cap() const { return cap_; }
  int nblocks() const { return nblocks_; }
  double timeout_s() const { return timeout_s_; }

 private:
  static hipStream_t stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

  void check(const at::Tensor& t, bool reduce) const {
    TORCH_CHECK(opened_ || world_ == 1, "OneShot: open() the peer workspaces first");
    TORCH_CHECK(t.is_cuda() && t.get_device() == device_, "OneShot: tensor on cuda:", device_);
    TORCH_CHECK(t.is_contiguous(), "OneShot: contiguous tensor");
    if (reduce) TORCH_CHECK(t.scalar_type() == at::kFloat, "OneShot: all_reduce is float32");
    const int64_t nb = t.numel() * t.element_size();
    TORCH_CHECK(nb % 16 == 0 && (uintptr_t)t.data_ptr() % 16 == 0,
                "OneShot: 16-byte aligned storage, size a multiple of 16 bytes");
    TORCH_CHECK(nb <= cap_, "OneShot: message of ", nb, " bytes exceeds the ", cap_,
                "-byte slot");
  }

  int rank_, world_;
  int64_t cap_;
  int device_;
  double timeout_s_;
  int nblocks_ = 1;
  char* own_ = nullptr;
  unsigned int* err_host_ = nullptr;  // pinned
  hipEvent_t err_ev_ = nullptr;
  bool requested_ = false;
  std::vector<char*> bases_;
  bool opened_ = false;
};

void init_oneshot(py::module& m) {
  py::class_<OneShot>(m, "OneShot")
      .def(py::init<int, int, int64_t, int, double>(), py::arg("rank"), py::arg("world"),
           py::arg("cap_bytes"), py::arg("device"), py::arg("timeout_s") = 120.0)
      .def("handle", &OneShot::handle)
      .def("open", &OneShot::open)
      .def("all_reduce", &OneShot::all_reduce, py::arg("t"), py::arg("avg") = false)
      .def("broadcast", &OneShot::broadcast, py::arg("t"), py::arg("src") = 0)
      .def("error", &OneShot::error)
      .def("error_info", &OneShot::error_info)
      .def("request_error", &OneShot::request_error)
      .def("poll_error", &OneShot::poll_error)
      .def_property_readonly("cap", &OneShot::cap)
      .def_property_readonly("nblocks", &OneShot::nblocks)
      .def_property_readonly("timeout_s", &OneShot::timeout_s);
}

}  // namespace mipipe_comm
