// Python registration of the native RCCL point-to-point engine (class in rccl_p2p.h).
#include "../comm/rccl_p2p.h"

namespace mipipe_comm {

void register_rccl(py::module& m) {
  py::class_<RcclP2P>(m, "RcclP2P")
      .def(py::init<const py::bytes&, int, int, int>(), py::arg("unique_ids"), py::arg("nranks"), py::arg("rank"),
           py::arg("device"))
      .def_static("load", &RcclP2P::load)
      .def_static("unique_id", &RcclP2P::unique_id)
      .def_static("id_bytes", &RcclP2P::id_bytes)
      .def("post", &RcclP2P::post, py::arg("channel"), py::arg("sends"), py::arg("recvs"))
      .def("wait", &RcclP2P::wait)
      .def("query", &RcclP2P::query)
      .def("synchronize", &RcclP2P::synchronize)
      .def("close", &RcclP2P::close)
      .def("abort", &RcclP2P::abort)
      .def("async_error", &RcclP2P::async_error)
      .def("stream_handle", &RcclP2P::stream_handle)
      .def_property_readonly("channels", &RcclP2P::channels)
      .def_property_readonly("rank", &RcclP2P::rank)
      .def_property_readonly("nranks", &RcclP2P::nranks);
}

}  // namespace mipipe_comm
