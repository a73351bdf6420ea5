// pybind11 bindings of the native runtime: module ``mipipe._runtime``.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime.hpp"

namespace py = pybind11;
using namespace mipipe_rt;

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "mipipe native runtime: process supervisor, DAG scheduler, record loader";

  py::class_<ProcessGroup>(m, "ProcessGroup")
      .def(py::init<bool>(), py::arg("echo") = true)
      .def("spawn", &ProcessGroup::spawn, py::arg("argv"), py::arg("env"), py::arg("cwd") = "",
           py::arg("log_path") = "", py::arg("prefix") = "")
      .def("wait", &ProcessGroup::wait, py::arg("timeout") = 0.0, py::arg("grace") = 10.0,
           py::call_guard<py::gil_scoped_release>())
      .def("signal_all", &ProcessGroup::signal_all)
      .def("interrupt", &ProcessGroup::interrupt)
      .def("exit_codes", &ProcessGroup::exit_codes)
      .def("pids", &ProcessGroup::pids)
      .def_property_readonly("failed_rank", &ProcessGroup::failed_rank);

  py::class_<DagScheduler> d(m, "DagScheduler");
  d.def(py::init<int, const std::vector<std::vector<int>>&, const std::vector<bool>&, bool>(),
        py::arg("n"), py::arg("deps"), py::arg("always_run"), py::arg("fail_fast") = true)
      .def("next_ready", &DagScheduler::next_ready)
      .def("complete", &DagScheduler::complete)
      .def("take_cancelled", &DagScheduler::take_cancelled)
      .def("mark_external_failure", &DagScheduler::mark_external_failure)
      .def("finished", &DagScheduler::finished)
      .def("deadlocked", &DagScheduler::deadlocked)
      .def("states", &DagScheduler::states)
      .def("topo_order", &DagScheduler::topo_order);
  d.attr("PENDING") = (int)DagScheduler::kPending;
  d.attr("RUNNING") = (int)DagScheduler::kRunning;
  d.attr("SUCCEEDED") = (int)DagScheduler::kSucceeded;
  d.attr("CACHED") = (int)DagScheduler::kCached;
  d.attr("SKIPPED") = (int)DagScheduler::kSkipped;
  d.attr("FAILED") = (int)DagScheduler::kFailed;
  d.attr("CANCELLED") = (int)DagScheduler::kCancelled;

  py::class_<LoaderConfig>(m, "LoaderConfig")
      .def(py::init<>())
      .def_readwrite("files", &LoaderConfig::files)
      .def_readwrite("header_bytes", &LoaderConfig::header_bytes)
      .def_readwrite("label_bytes", &LoaderConfig::label_bytes)
      .def_readwrite("C", &LoaderConfig::C)
      .def_readwrite("H", &LoaderConfig::H)
      .def_readwrite("W", &LoaderConfig::W)
      .def_readwrite("batch", &LoaderConfig::batch)
      .def_readwrite("train", &LoaderConfig::train)
      .def_readwrite("pad", &LoaderConfig::pad)
      .def_readwrite("flip", &LoaderConfig::flip)
      .def_readwrite("mean", &LoaderConfig::mean)
      .def_readwrite("std", &LoaderConfig::stdv)
      .def_readwrite("seed", &LoaderConfig::seed)
      .def_readwrite("workers", &LoaderConfig::workers)
      .def_readwrite("prefetch", &LoaderConfig::prefetch)
      .def_readwrite("drop_last", &LoaderConfig::drop_last);

  py::class_<RecordLoader>(m, "RecordLoader")
      .def(py::init<const LoaderConfig&>())
      .def("__len__", &RecordLoader::size)
      .def("size", &RecordLoader::size)
      .def("start_epoch", &RecordLoader::start_epoch, py::call_guard<py::gil_scoped_release>())
      .def("batches_per_epoch", &RecordLoader::batches_per_epoch)
      // x_ptr / y_ptr: addresses of caller-owned (pinned) host buffers large enough for a batch
      .def("next_into",
           [](RecordLoader& l, uintptr_t x, uintptr_t y) {
             return l.next(reinterpret_cast<float*>(x), reinterpret_cast<int64_t*>(y));
           },
           py::call_guard<py::gil_scoped_release>());
}
