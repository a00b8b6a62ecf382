// Binding for the one-shot / two-shot IPC all-reduce (csrc/kernels/allreduce.hip):
// operator_amd._C.CustomAllReduce. The handle exchange itself happens in
// Python over the process group (operator_amd/parallel/custom_ar.py); this
// object owns the local fine-grained buffer and the opened peer mappings.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <string>
#include <vector>

#include "kernels/kernels.h"

namespace {

class CustomAllReduce {
 public:
  CustomAllReduce(int64_t cap_bytes, int64_t rank, int64_t world, int64_t blocks, int64_t device, double timeout_s)
      : cap_(cap_bytes), rank_(rank), world_(world), blocks_(blocks), device_(device), timeout_s_(timeout_s) {
    TORCH_CHECK(world >= 1 && world <= 8, "CustomAllReduce: world must be 1..8");
    TORCH_CHECK(rank >= 0 && rank < world, "CustomAllReduce: bad rank");
    TORCH_CHECK(cap_bytes > 0 && cap_bytes % 16 == 0, "CustomAllReduce: capacity must be a positive multiple of 16 B");
    TORCH_CHECK(blocks >= 1 && blocks <= 64, "CustomAllReduce: blocks must be 1..64");
    const c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
    char h[64];
    const int rc = oamd::car_alloc((size_t)cap_bytes, (int)world, &base_, h);
    TORCH_CHECK(rc == 0, "CustomAllReduce: buffer allocation / IPC export failed rc=", rc);
    handle_.assign(h, 64);
    TORCH_CHECK(oamd::car_host_flag(&herr_, &herr_dev_) == 0, "CustomAllReduce: host-mapped error word failed");
    bases_.assign(world, nullptr);
    bases_[rank] = base_;
  }
  ~CustomAllReduce() { close(); }

  pybind11::bytes handle() const { return pybind11::bytes(handle_); }

  void open(const std::vector<std::string>& handles) {
    TORCH_CHECK((int64_t)handles.size() == world_, "CustomAllReduce.open: need one handle per rank");
    const c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    for (int64_t p = 0; p < world_; ++p) {
      if (p == rank_) continue;
      TORCH_CHECK(handles[p].size() == 64, "CustomAllReduce.open: handle of rank ", p, " is not 64 bytes");
      void* ptr = nullptr;
      const int rc = oamd::car_open(handles[p].data(), &ptr);
      TORCH_CHECK(rc == 0, "CustomAllReduce.open: hipIpcOpenMemHandle of rank ", p, " failed rc=", rc);
      bases_[p] = ptr;
    }
    opened_ = true;
  }

  // proto: 0 one-shot, 1 two-shot (reduce-scatter + all-gather), 2 one-shot with the original
  // system-fence hand-off (A/B)
  void all_reduce(const at::Tensor& in, at::Tensor& out, int64_t proto) {
    TORCH_CHECK(opened_ || world_ == 1, "CustomAllReduce: open() the peer handles first");
    TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.device().index() == device_, "tensors must be on this device");
    TORCH_CHECK(in.is_contiguous() && out.is_contiguous(), "tensors must be contiguous");
    TORCH_CHECK(in.scalar_type() == out.scalar_type() && in.numel() == out.numel(), "in/out mismatch");
    TORCH_CHECK(in.scalar_type() == at::kBFloat16 || in.scalar_type() == at::kFloat, "dtype must be bf16 or fp32");
    const int64_t bytes = in.numel() * in.element_size();
    TORCH_CHECK(bytes % 16 == 0 && bytes <= cap_, "size must be a multiple of 16 B and <= capacity");
    const c10::hip::HIPGuardMasqueradingAsCUDA g(in.device());
    const int rc = oamd::car_all_reduce(in.data_ptr(), out.data_ptr(), bytes, in.scalar_type() == at::kBFloat16,
                                        (int)rank_, (int)world_, bases_.data(), (size_t)cap_, (int)blocks_,
                                        herr_dev_, timeout_s_, (int)proto,
                                        c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
    TORCH_CHECK(rc == 0, "IPC all-reduce launch failed rc=", rc);
  }

  // residual += all_reduce(in) (bf16-rounded); y = rmsnorm(residual) * w — one launch.
  // `in` = None with `slabs` = S fp32 split-K slabs of the producing GEMM (summed in the kernel);
  // q8/sx given: y is also emitted as per-row e4m3fn for the next fp8 GEMM.
  void all_reduce_rmsnorm(const c10::optional<at::Tensor>& in, at::Tensor& residual, const at::Tensor& w,
                          at::Tensor& y, double eps, const c10::optional<at::Tensor>& slabs, int64_t splits,
                          const c10::optional<at::Tensor>& q8, const c10::optional<at::Tensor>& sx, int64_t proto) {
    TORCH_CHECK(opened_ || world_ == 1, "CustomAllReduce: open() the peer handles first");
    TORCH_CHECK(in.has_value() != slabs.has_value(), "exactly one of in / slabs");
    TORCH_CHECK(q8.has_value() == sx.has_value(), "q8 and sx together");
    auto on_dev = [&](const at::Tensor& t) {
      TORCH_CHECK(t.is_cuda() && t.device().index() == device_ && t.is_contiguous(), "contiguous tensors on this device");
    };
    for (const at::Tensor* t : {const_cast<const at::Tensor*>(&residual), &w, const_cast<const at::Tensor*>(&y)}) {
      on_dev(*t);
      TORCH_CHECK(t->scalar_type() == at::kBFloat16, "bf16 residual / w / y");
    }
    TORCH_CHECK(residual.dim() == 2 && y.sizes() == residual.sizes(), "[rows, hidden] shapes");
    const int64_t rows = residual.size(0), hidden = residual.size(1);
    TORCH_CHECK(w.numel() == hidden, "w [hidden]");
    TORCH_CHECK(hidden % 8 == 0 && hidden <= 16384, "hidden % 8 == 0 and <= 16384");
    TORCH_CHECK(rows * hidden * 2 <= cap_, "size must be <= capacity");
    const void* ip = nullptr;
    const float* sp = nullptr;
    if (in.has_value()) {
      on_dev(*in);
      TORCH_CHECK(in->scalar_type() == at::kBFloat16 && in->sizes() == residual.sizes(), "in: bf16 [rows, hidden]");
      ip = in->data_ptr();
    } else {
      on_dev(*slabs);
      TORCH_CHECK(slabs->scalar_type() == at::kFloat && splits >= 1 && slabs->numel() >= splits * rows * hidden,
                  "slabs: fp32 [splits, rows, hidden]");
      sp = slabs->data_ptr<float>();
    }
    uint8_t* qp = nullptr;
    float* xp = nullptr;
    if (q8.has_value()) {
      on_dev(*q8);
      on_dev(*sx);
      TORCH_CHECK((q8->scalar_type() == at::kByte || q8->scalar_type() == at::kFloat8_e4m3fn) &&
                      q8->numel() == rows * hidden && sx->scalar_type() == at::kFloat && sx->numel() == rows,
                  "q8 e4m3fn [rows, hidden], sx fp32 [rows]");
      qp = static_cast<uint8_t*>(q8->data_ptr());
      xp = sx->data_ptr<float>();
    }
    const c10::hip::HIPGuardMasqueradingAsCUDA g(residual.device());
    const int rc = oamd::car_all_reduce_rmsnorm(
        ip, sp, (int)splits, reinterpret_cast<oamd::bf16_t*>(residual.data_ptr()),
        reinterpret_cast<const oamd::bf16_t*>(w.data_ptr()), reinterpret_cast<oamd::bf16_t*>(y.data_ptr()), qp, xp,
        (int)rows, (int)hidden, (float)eps, (int)rank_, (int)world_, bases_.data(), (size_t)cap_, (int)blocks_,
        herr_dev_, timeout_s_, (int)proto, c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
    TORCH_CHECK(rc == 0, "IPC all-reduce + rmsnorm launch failed rc=", rc);
  }

  // Host read of the mapped error word: no device synchronisation, so the engine
  // can poll it after every decode window without draining its pipelined windows.
  int64_t error() const { return herr_ != nullptr ? oamd::car_error(herr_) : 0; }

  // Collective: every rank, between two barriers, with no call in flight.
  void reset() {
    TORCH_CHECK(base_ != nullptr, "CustomAllReduce: closed");
    const c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    TORCH_CHECK(oamd::car_reset(base_, oamd::car_buffer_bytes((size_t)cap_, (int)world_), herr_) == 0, "CustomAllReduce.reset failed");
  }

  void close() {
    if (base_ == nullptr) return;
    const c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    (void)hipDeviceSynchronize();
    for (int64_t p = 0; p < world_; ++p)
      if (p != rank_ && bases_[p] != nullptr) (void)oamd::car_close(bases_[p]);
    (void)oamd::car_free(base_);
    oamd::car_free_host_flag(herr_);
    herr_ = nullptr;
    herr_dev_ = nullptr;
    base_ = nullptr;
    bases_.assign(world_, nullptr);
    opened_ = false;
  }

  int64_t capacity() const { return cap_; }

 private:
  int64_t cap_, rank_, world_, blocks_, device_;
  double timeout_s_;
  void* base_ = nullptr;
  uint32_t* herr_ = nullptr;
  uint32_t* herr_dev_ = nullptr;
  std::string handle_;
  std::vector<void*> bases_;
  bool opened_ = false;
};

}  // namespace

void register_comm_bindings(pybind11::module_& m) {
  pybind11::class_<CustomAllReduce>(m, "CustomAllReduce")
      .def(pybind11::init<int64_t, int64_t, int64_t, int64_t, int64_t, double>(), pybind11::arg("cap_bytes"),
           pybind11::arg("rank"), pybind11::arg("world"), pybind11::arg("blocks"), pybind11::arg("device"),
           pybind11::arg("timeout_s") = 2.0)
      .def("handle", &CustomAllReduce::handle)
      .def("open", &CustomAllReduce::open)
      .def("all_reduce", &CustomAllReduce::all_reduce, pybind11::arg("in"), pybind11::arg("out"),
           pybind11::arg("proto") = 0)
      .def("all_reduce_rmsnorm", &CustomAllReduce::all_reduce_rmsnorm, pybind11::arg("in"), pybind11::arg("residual"),
           pybind11::arg("w"), pybind11::arg("y"), pybind11::arg("eps"), pybind11::arg("slabs") = pybind11::none(),
           pybind11::arg("splits") = 1, pybind11::arg("q8") = pybind11::none(), pybind11::arg("sx") = pybind11::none(),
           pybind11::arg("proto") = 0)
      .def("error", &CustomAllReduce::error)
      .def("reset", &CustomAllReduce::reset)
      .def("close", &CustomAllReduce::close)
      .def_property_readonly("capacity", &CustomAllReduce::capacity);
}
