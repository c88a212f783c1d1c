// pybind11 module cloud_amd._monitoring: the Python face of the native metrics
// library (registry writes from the training loop / launcher / tuner, and the
// periodic exporter with a JSONL or Prometheus-textfile sink).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "metrics.h"

namespace py = pybind11;
using namespace cloud_amd::monitoring;

namespace {
std::unique_ptr<Exporter> g_exporter;
std::shared_ptr<RecordingSink> g_recorder;

py::dict DistToDict(const Distribution& d) {
  py::dict o;
  o["count"] = d.count;
  o["mean"] = d.mean;
  o["sum_of_squared_deviation"] = d.sum_of_squared_deviation;
  o["bounds"] = d.bounds;
  o["bucket_counts"] = d.bucket_counts;
  return o;
}
}  // namespace

PYBIND11_MODULE(_monitoring, m) {
  m.doc() = "cloud_amd native metrics registry + exporter";
  m.def("define", [](const std::string& name, const std::string& desc, const std::string& kind,
                     const std::string& vtype, const std::vector<std::string>& labels) {
    MetricDescriptor d;
    d.name = name;
    d.description = desc;
    d.label_names = labels;
    d.kind = kind == "gauge" ? MetricKind::kGauge : MetricKind::kCumulative;
    d.value_type = vtype == "histogram" ? ValueType::kHistogram
                   : vtype == "double" ? ValueType::kDouble
                   : vtype == "string" ? ValueType::kString
                   : vtype == "bool"   ? ValueType::kBool
                                       : ValueType::kInt64;
    MetricRegistry::Default()->Define(d);
  }, py::arg("name"), py::arg("description") = "", py::arg("kind") = "cumulative", py::arg("value_type") = "int64",
     py::arg("labels") = std::vector<std::string>{});
  m.def("counter_inc", [](const std::string& n, int64_t d, const Labels& l) {
    MetricRegistry::Default()->IncrementCounter(n, d, l);
  }, py::arg("name"), py::arg("delta") = 1, py::arg("labels") = Labels{});
  m.def("gauge_set", [](const std::string& n, double v, const Labels& l) { MetricRegistry::Default()->SetGauge(n, v, l); },
        py::arg("name"), py::arg("value"), py::arg("labels") = Labels{});
  m.def("observe", [](const std::string& n, double v, const Labels& l, const std::vector<double>& b) {
    MetricRegistry::Default()->Observe(n, v, l, b);
  }, py::arg("name"), py::arg("value"), py::arg("labels") = Labels{}, py::arg("bounds") = std::vector<double>{});
  m.def("clear", [] { MetricRegistry::Default()->Clear(); });
  m.def("snapshot", [] {
    py::dict out;
    auto c = MetricRegistry::Default()->Collect();
    for (const auto& kv : c.point_sets) {
      py::list pts;
      for (const auto& p : kv.second->points) {
        py::dict d;
        d["labels"] = p->labels;
        TimeSeriesPoint tp;
        ConvertPoint(*p, &tp);
        switch (p->value_type) {
          case ValueType::kInt64: d["value"] = p->int64_value; break;
          case ValueType::kDouble: d["value"] = p->double_value; break;
          case ValueType::kString: d["value"] = p->string_value; break;
          case ValueType::kBool: d["value"] = p->bool_value; break;
          case ValueType::kHistogram: d["value"] = DistToDict(tp.distribution); break;
        }
        pts.append(d);
      }
      out[py::str(kv.first)] = pts;
    }
    return out;
  });
  m.def("convert_distribution", [](const std::vector<double>& values, const std::vector<double>& bounds) {
    Histogram h = Histogram::WithBounds(bounds);
    for (double v : values) h.Add(v);
    Distribution d;
    ConvertDistribution(h, &d);
    return DistToDict(d);
  });
  m.def("start_exporter", [](const std::string& dir, const std::string& sink, double interval_s, bool force) {
    ExporterConfig cfg = ExporterConfig::FromEnv();
    if (force) cfg.enabled = true;
    if (interval_s > 0) cfg.interval_millis = (int64_t)(interval_s * 1000);
    std::shared_ptr<MetricSink> s;
    if (sink == "prometheus") s = std::make_shared<PrometheusTextSink>(dir + "/metrics.prom");
    else if (sink == "memory") { g_recorder = std::make_shared<RecordingSink>(); s = g_recorder; }
    else s = std::make_shared<JsonlFileSink>(dir);
    if (g_exporter) g_exporter->Stop();
    g_exporter = std::make_unique<Exporter>(MetricRegistry::Default(), s, cfg);
    return g_exporter->PeriodicallyExportMetrics();
  }, py::arg("dir"), py::arg("sink") = "jsonl", py::arg("interval_s") = 0.0, py::arg("force") = false);
  m.def("export_now", [] { if (g_exporter) g_exporter->ExportMetrics(); });
  m.def("stop_exporter", [] { if (g_exporter) { g_exporter->ExportMetrics(); g_exporter->Stop(); g_exporter.reset(); } });
  m.def("exports", [] { return g_exporter ? g_exporter->exports() : 0; });
  m.def("config_debug_string", [] { return ExporterConfig::FromEnv().DebugString(); });
  m.def("recorded_series", [] {
    py::list out;
    if (!g_recorder) return out;
    std::lock_guard<std::mutex> l(g_recorder->mu);
    for (const auto& r : g_recorder->series_requests)
      for (const auto& ts : r.time_series) out.append(TimeSeriesToJson(ts));
    return out;
  });
}
