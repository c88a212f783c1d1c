// Python bindings of the native input pipeline (csrc/data/loader_core.h): the
// blocking calls release the GIL so the C++ workers and the training thread overlap.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "loader_core.h"

namespace py = pybind11;
using ca_data::Loader;
using ca_data::NpyArray;
using ca_data::open_npy;

PYBIND11_MODULE(_data, m) {
  m.doc() = "cloud_amd native input pipeline: mmap'd .npy arrays -> sharded, shuffled batches (C++ workers)";
  m.def("npy_info", [](const std::string& path) {
    NpyArray a = open_npy(path);
    py::dict d;
    d["descr"] = a.descr;
    d["shape"] = a.shape;
    d["row_bytes"] = a.row_bytes;
    munmap(a.map, a.map_bytes);
    return d;
  });
  py::class_<Loader>(m, "Loader")
      .def(py::init<const std::vector<std::string>&, long, bool, uint64_t, int, int, bool, int,
                    const std::vector<std::vector<uint64_t>>&>(),
           py::arg("paths"), py::arg("batch"), py::arg("shuffle"), py::arg("seed"), py::arg("rank"), py::arg("world"),
           py::arg("drop_remainder"), py::arg("threads"), py::arg("slots"))
      .def("start_epoch", &Loader::start_epoch, py::call_guard<py::gil_scoped_release>())
      .def("next", &Loader::next, py::call_guard<py::gil_scoped_release>())
      .def("release", &Loader::release)
      .def("num_samples", &Loader::num_samples)
      .def("arrays_info", [](const Loader& l) {
        py::list out;
        for (const auto& a : l.arrays()) {
          py::dict d;
          d["path"] = a.path;
          d["descr"] = a.descr;
          d["shape"] = a.shape;
          d["row_bytes"] = a.row_bytes;
          out.append(d);
        }
        return out;
      });
}
