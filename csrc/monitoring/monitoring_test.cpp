// Golden tests for the native metrics library (parity with reference
// src/cpp/monitoring/stackdriver_client_test.cc, against a recording sink
// instead of a gRPC mock stub).  Build: python -c "from cloud_amd import _build;
// print(_build.build_monitoring_test())"; run the printed binary.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "metrics.h"

using namespace cloud_amd::monitoring;

static int g_failures = 0;
#define CHECK(cond)                                                              \
  do {                                                                           \
    if (!(cond)) {                                                               \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
      ++g_failures;                                                              \
    }                                                                            \
  } while (0)
#define CHECK_NEAR(a, b) CHECK(std::fabs((double)(a) - (double)(b)) < 1e-9)

static void TestCreateTimeSeriesInt64FirstPoint() {
  PointSet ps;
  ps.metric_name = "/metric_1";
  auto p1 = std::make_unique<Point>();
  p1->value_type = ValueType::kInt64;
  p1->int64_value = 7;
  p1->end_timestamp_millis = 1000;
  auto p2 = std::make_unique<Point>();
  p2->int64_value = 9;
  ps.points.push_back(std::move(p1));
  ps.points.push_back(std::move(p2));
  TimeSeries ts;
  ConvertPointSet(ps, &ts);
  CHECK(ts.metric_type == std::string(kMetricTypePrefix) + "/metric_1");
  CHECK(ts.resource_type == "global");
  CHECK(ts.points.size() == 1);
  CHECK(ts.points[0].int64_value == 7);
  CHECK(ts.points[0].end_time_millis == 1000);
}

static void TestHistogramDistributionMath() {
  Histogram h = Histogram::WithBounds({0.0});
  h.Add(-1.0);
  h.Add(1.0);
  Distribution d;
  ConvertDistribution(h, &d);
  CHECK(d.count == 2);
  CHECK_NEAR(d.mean, 0.0);
  CHECK_NEAR(d.sum_of_squared_deviation, 2.0);
  CHECK(d.bounds.size() == 1 && d.bounds[0] == 0.0);
  CHECK(d.bucket_counts.size() == 2 && d.bucket_counts[0] == 1 && d.bucket_counts[1] == 1);
  Histogram e = Histogram::WithBounds({1.0, 2.0});
  Distribution de;
  ConvertDistribution(e, &de);
  CHECK(de.count == 0 && de.mean == 0.0 && de.sum_of_squared_deviation == 0.0);
}

static void TestDescriptorType() {
  MetricDescriptor md;
  md.name = "metric_1";
  md.kind = MetricKind::kCumulative;
  md.value_type = ValueType::kInt64;
  const std::string js = DescriptorToJson(md, std::string(kMetricTypePrefix) + md.name);
  // the prefix is concatenated without a '/', as in the reference (custom.googleapis.commetric_1)
  CHECK(js.find("\"type\":\"custom.cloud_amdmetric_1\"") != std::string::npos);
  CHECK(js.find("\"metricKind\":\"CUMULATIVE\"") != std::string::npos);
}

static void TestExporterFilterAndDescriptorOnce() {
  MetricRegistry reg;
  reg.IncrementCounter("/cloud_amd/launcher/jobs", 2, {{"state", "ok"}});
  reg.IncrementCounter("/not/whitelisted", 5);
  reg.IncrementCounter("/cloud_amd/tuner/trials", 0);  // zero -> not exported
  reg.Observe("/cloud_amd/train/step_time_ms", 33.0);
  ExporterConfig cfg;
  cfg.enabled = true;
  cfg.project_id = "p";
  cfg.whitelist = {"/cloud_amd/launcher/jobs", "/cloud_amd/tuner/trials", "/cloud_amd/train/step_time_ms"};
  auto sink = std::make_shared<RecordingSink>();
  sink->existing.insert(std::string(kMetricTypePrefix) + "/cloud_amd/train/step_time_ms");
  Exporter ex(&reg, sink, cfg);
  ex.ExportMetrics();
  ex.ExportMetrics();
  CHECK(sink->series_requests.size() == 2);
  CHECK(sink->series_requests[0].name == "projects/p");
  CHECK(sink->series_requests[0].time_series.size() == 2);
  CHECK(sink->descriptor_types.size() == 2);  // once per metric, ALREADY_EXISTS counts as success
}

static void TestPeriodicExport() {
  MetricRegistry reg;
  reg.IncrementCounter("/cloud_amd/launcher/jobs", 1);
  ExporterConfig cfg;
  cfg.enabled = true;
  cfg.whitelist = {"/cloud_amd/launcher/jobs"};
  cfg.interval_millis = 10;
  auto sink = std::make_shared<RecordingSink>();
  Exporter ex(&reg, sink, cfg);
  CHECK(ex.PeriodicallyExportMetrics());
  CHECK(ex.PeriodicallyExportMetrics());  // idempotent
  for (int i = 0; i < 200 && ex.exports() < 3; ++i) {
    struct timespec t = {0, 5 * 1000 * 1000};
    nanosleep(&t, nullptr);
  }
  ex.Stop();
  CHECK(ex.exports() >= 3);
  ExporterConfig off;
  Exporter disabled(&reg, sink, off);
  CHECK(!disabled.PeriodicallyExportMetrics());
}

static void TestConfigFromEnv() {
  setenv("CLOUD_AMD_MONITORING_METRICS_WHITELIST", "/a,/b", 1);
  setenv("CLOUD_AMD_MONITORING_EXPORTER_ENABLED", "true", 1);
  ExporterConfig c = ExporterConfig::FromEnv();
  CHECK(c.enabled && c.IsWhitelisted("/a") && c.IsWhitelisted("/b") && !c.IsWhitelisted("/c"));
  unsetenv("CLOUD_AMD_MONITORING_METRICS_WHITELIST");
  unsetenv("CLOUD_AMD_MONITORING_EXPORTER_ENABLED");
  ExporterConfig d = ExporterConfig::FromEnv();
  CHECK(!d.enabled && d.IsWhitelisted("/cloud_amd/train/step_time_ms"));
}

int main() {
  TestCreateTimeSeriesInt64FirstPoint();
  TestHistogramDistributionMath();
  TestDescriptorType();
  TestExporterFilterAndDescriptorOnce();
  TestPeriodicExport();
  TestConfigFromEnv();
  if (g_failures) {
    std::fprintf(stderr, "%d check(s) failed\n", g_failures);
    return 1;
  }
  std::printf("monitoring_test: all checks passed\n");
  return 0;
}
