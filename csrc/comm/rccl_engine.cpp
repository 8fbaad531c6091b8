// Python registration of the native RCCL engine (class in rccl_engine.h) and of the comm
// stream slots (parallel/queues.py probes them).
#include "../comm/rccl_engine.h"

namespace mipipe_comm {

void register_rccl(py::module& m) {
  py::class_<RcclEngine>(m, "RcclEngine")
      .def(py::init<const py::bytes&, int, int, int, std::vector<int64_t>>(), py::arg("unique_ids"),
           py::arg("nranks"), py::arg("rank"), py::arg("device"), py::arg("slots"))
      .def_static("load", &RcclEngine::load)
      .def_static("unique_id", &RcclEngine::unique_id)
      .def_static("id_bytes", &RcclEngine::id_bytes)
      .def("post", &RcclEngine::post, py::arg("channel"), py::arg("sends"), py::arg("recvs"))
      .def("coll", &RcclEngine::coll, py::arg("channel"), py::arg("op"), py::arg("send"), py::arg("recv"))
      .def("wait", &RcclEngine::wait)
      .def("wait_keep", &RcclEngine::wait_keep)
      .def("release", &RcclEngine::release)
      .def("query", &RcclEngine::query)
      .def("synchronize", &RcclEngine::synchronize)
      .def("close", &RcclEngine::close)
      .def("abort", &RcclEngine::abort)
      .def("async_error", &RcclEngine::async_error)
      .def("progress", &RcclEngine::progress)
      .def("issued", &RcclEngine::issued)
      .def("stream_handle", &RcclEngine::stream_handle)
      .def("slot", &RcclEngine::slot)
      .def_property_readonly("channels", &RcclEngine::channels)
      .def_property_readonly("rank", &RcclEngine::rank)
      .def_property_readonly("nranks", &RcclEngine::nranks);
  m.def("comm_stream", [](int device, int slot) { return reinterpret_cast<int64_t>(comm_stream(device, slot)); },
        py::arg("device"), py::arg("slot"));
  m.attr("COMM_STREAM_SLOTS") = kStreamSlots;
}

}  // namespace mipipe_comm
