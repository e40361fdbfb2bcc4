// torch bindings of the native communication engine
// (module `ray_lightning_accelerators_amd._comm`).
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "comm/communicator.h"
#include "comm/fusion_engine.h"
#include "comm/reducer.h"

namespace {

using at::Tensor;
using rla::comm::Communicator;
using rla::comm::DType;
using rla::comm::FusionEngine;
using rla::comm::RedOp;
using rla::comm::Reducer;

hipStream_t cur_stream(const Tensor& t) {
  return at::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.get_device()).stream();
}

DType dtype_of(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return DType::kF32;
    case at::kBFloat16: return DType::kBF16;
    case at::kHalf: return DType::kF16;
    case at::kInt: return DType::kI32;
    case at::kLong: return DType::kI64;
    case at::kByte: return DType::kU8;
    case at::kDouble: return DType::kF64;
    default: TORCH_CHECK(false, "unsupported dtype for collectives: ", t.scalar_type());
  }
}

void check(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "Native comm engine: RCCL communicator, xGMI one-shot allreduce, fusion engine";
  py::class_<Communicator>(m, "Communicator")
      .def(py::init<int, int, int>(), py::arg("rank"), py::arg("world"), py::arg("device"))
      .def_static("unique_id", []() { return py::bytes(Communicator::unique_id()); })
      .def("init_rccl",
           [](Communicator& c, py::bytes uid) {
             const std::string id(uid);  // copy while holding the GIL
             py::gil_scoped_release nogil;
             c.init_rccl(id);
           })
      .def_property_readonly("rank", &Communicator::rank)
      .def_property_readonly("world", &Communicator::world)
      .def_property_readonly("has_rccl", &Communicator::has_rccl)
      .def_property_readonly("rccl_count", &Communicator::rccl_count)
      .def_property_readonly("has_xgmi", &Communicator::has_xgmi)
      .def_property_readonly("xgmi_capacity", &Communicator::xgmi_capacity)
      .def("allreduce",
           [](Communicator& c, Tensor t, int op) {
             check(t, "tensor");
             c.allreduce(t.data_ptr(), t.numel(), dtype_of(t), static_cast<RedOp>(op), cur_stream(t));
           },
           py::arg("tensor"), py::arg("op") = 0)
      .def("broadcast",
           [](Communicator& c, Tensor t, int root) {
             check(t, "tensor");
             c.broadcast(t.data_ptr(), t.numel(), dtype_of(t), root, cur_stream(t));
           })
      .def("allgather",
           [](Communicator& c, Tensor in, Tensor out) {
             check(in, "input");
             check(out, "output");
             TORCH_CHECK(out.numel() == in.numel() * c.world() && out.scalar_type() == in.scalar_type(),
                         "allgather output must hold world * input elements of the same dtype");
             c.allgather(in.data_ptr(), out.data_ptr(), in.numel(), dtype_of(in), cur_stream(in));
           })
      .def("reduce_scatter",
           [](Communicator& c, Tensor in, Tensor out, int op) {
             check(in, "input");
             check(out, "output");
             TORCH_CHECK(in.numel() == out.numel() * c.world() && out.scalar_type() == in.scalar_type(),
                         "reduce_scatter input must hold world * output elements of the same dtype");
             c.reduce_scatter(in.data_ptr(), out.data_ptr(), out.numel(), dtype_of(in), static_cast<RedOp>(op),
                              cur_stream(in));
           },
           py::arg("input"), py::arg("output"), py::arg("op") = 0)
      .def("xgmi_handle", [](Communicator& c, int64_t cap) { return py::bytes(c.xgmi_handle(cap)); })
      .def("xgmi_open",
           [](Communicator& c, std::vector<py::bytes> hs) {
             std::vector<std::string> v;
             for (auto& h : hs) v.emplace_back(std::string(h));
             c.xgmi_open(v);
           })
      .def("allreduce_xgmi",
           [](Communicator& c, Tensor t) {
             check(t, "tensor");
             TORCH_CHECK(t.scalar_type() == at::kFloat, "xGMI one-shot allreduce is fp32");
             c.allreduce_xgmi(t.data_ptr<float>(), t.numel(), cur_stream(t));
           })
      .def("twoshot_handle", [](Communicator& c, int64_t cap) { return py::bytes(c.twoshot_handle(cap)); })
      .def("twoshot_open",
           [](Communicator& c, std::vector<py::bytes> hs) {
             std::vector<std::string> v;
             for (auto& h : hs) v.emplace_back(std::string(h));
             c.twoshot_open(v);
           })
      .def_property_readonly("has_twoshot", &Communicator::has_twoshot)
      .def_property_readonly("twoshot_capacity", &Communicator::twoshot_capacity)
      .def("allreduce_twoshot",
           [](Communicator& c, Tensor t, bool bf16_wire) {
             check(t, "tensor");
             TORCH_CHECK(t.scalar_type() == at::kFloat, "xGMI two-shot allreduce takes fp32 buckets");
             c.allreduce_twoshot(t.data_ptr<float>(), t.numel(), bf16_wire, cur_stream(t));
           },
           py::arg("tensor"), py::arg("bf16_wire") = false)
      .def("set_route_limits", &Communicator::set_route_limits, py::arg("oneshot_max_floats"),
           py::arg("twoshot_max_floats"))
      .def("route",
           [](Communicator& c, Tensor t) {
             check(t, "tensor");
             return c.route(t.data_ptr<float>(), t.numel());
           })
      .def("allreduce_f32",
           [](Communicator& c, Tensor t) {
             check(t, "tensor");
             TORCH_CHECK(t.scalar_type() == at::kFloat, "allreduce_f32 takes fp32 tensors");
             c.allreduce_f32(t.data_ptr<float>(), t.numel(), cur_stream(t));
           })
      .def("allreduce_bf16wire",
           [](Communicator& c, Tensor t) {
             check(t, "tensor");
             TORCH_CHECK(t.scalar_type() == at::kFloat, "bf16-wire allreduce takes fp32 tensors");
             return c.allreduce_f32_bf16wire(t.data_ptr<float>(), t.numel(), cur_stream(t));
           })
      .def("aux_handle", [](Communicator& c, int64_t cap) { return py::bytes(c.aux_handle(cap)); })
      .def("aux_open",
           [](Communicator& c, std::vector<py::bytes> hs) {
             std::vector<std::string> v;
             for (auto& h : hs) v.emplace_back(std::string(h));
             c.aux_open(v);
           })
      .def_property_readonly("has_aux", &Communicator::has_aux)
      .def("aux_context", &Communicator::aux_context)
      .def("aux_rearm", &Communicator::aux_rearm)
      .def("set_spin_limit", &Communicator::set_spin_limit)
      .def("error_state", &Communicator::error_state)
      .def("error_message", &Communicator::error_message)
      .def("reset_error", &Communicator::reset_error)
      .def("disable_path", &Communicator::disable_path)
      .def("start_watchdog", &Communicator::start_watchdog, py::arg("period_ms") = 100)
      .def("abort", &Communicator::abort);

  py::class_<FusionEngine>(m, "FusionEngine")
      .def(py::init<Communicator*, int64_t, int>(), py::arg("comm"), py::arg("fusion_bytes"), py::arg("device"),
           py::keep_alive<1, 2>())
      .def("submit",
           [](FusionEngine& e, Tensor t, double scale) {
             check(t, "tensor");
             TORCH_CHECK(t.scalar_type() == at::kFloat, "fusion engine tensors are fp32");
             return e.submit(t.data_ptr<float>(), t.numel(), (float)scale, cur_stream(t));
           },
           py::arg("tensor"), py::arg("postscale") = 1.0)
      .def("flush", &FusionEngine::flush)
      .def("wait",
           [](FusionEngine& e, int64_t h, Tensor like) { return e.wait(h, cur_stream(like)); },
           py::call_guard<py::gil_scoped_release>())
      .def("drain", &FusionEngine::drain, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("fingerprint", &FusionEngine::fingerprint)
      .def_property_readonly("batches_executed", &FusionEngine::batches_executed)
      .def("last_error", &FusionEngine::last_error);
  py::class_<Reducer>(m, "Reducer")
      .def(py::init([](Communicator* c, Tensor grad, std::vector<int64_t> bounds, std::vector<int> pb, int dev) {
             check(grad, "grad arena");
             TORCH_CHECK(grad.scalar_type() == at::kFloat, "gradient arena must be fp32");
             return new Reducer(c, grad.data_ptr<float>(), grad.numel(), bounds, pb, dev);
           }),
           py::arg("comm"), py::arg("grad"), py::arg("bucket_bounds"), py::arg("param_bucket"), py::arg("device"),
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>())
      .def("prepare", &Reducer::prepare)
      .def("mark_ready", [](Reducer& r, int i, Tensor like) { r.mark_ready(i, cur_stream(like)); })
      .def("finish", [](Reducer& r, Tensor like) { r.finish(cur_stream(like)); })
      .def_property_readonly("launched", &Reducer::launched)
      .def_property_readonly("num_buckets", &Reducer::num_buckets);
  m.attr("XGMI_MAX_RANKS") = rla::comm::kXgmiMaxRanks;
  m.attr("ARCH") = "gfx950";
}
