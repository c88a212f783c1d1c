// cloud_amd native metrics: registry, value model, exporter and sinks.
//
// MI355X-native replacement for the reference's TensorFlow-plugin Stackdriver
// exporter (src/cpp/monitoring/stackdriver_{exporter,client,config}.{h,cc}):
//
//   * MetricRegistry  -- thread-safe counters / gauges / histograms with labels,
//                        fed by the launcher, the DP engine, the training loop
//                        and the tuner (stands in for TF's CollectionRegistry);
//   * ExporterConfig  -- env switches + metric allow-list (stackdriver_config.cc);
//   * Converter       -- PointSet -> time-series records, with the reference's
//                        histogram -> distribution math (stackdriver_client.cc:69-98);
//   * MetricSink      -- where records go: JSONL file, Prometheus textfile, or a
//                        recording mock for golden tests (replaces the gRPC stub);
//   * Exporter        -- a periodic background thread (default 10 s), idempotent
//                        start, "descriptor once" bookkeeping, whitelist + non-empty
//                        filtering (stackdriver_exporter.cc:38-126).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace cloud_amd {
namespace monitoring {

enum class MetricKind { kCumulative, kGauge };
enum class ValueType { kInt64, kDouble, kString, kBool, kHistogram };

using Labels = std::map<std::string, std::string>;

struct Histogram {
  // bucket_limits[i] is the upper bound of bucket i; the last is +inf (TF convention).
  std::vector<double> bucket_limits;
  std::vector<double> bucket_counts;
  double num = 0, sum = 0, sum_squares = 0, min = 0, max = 0;

  static Histogram WithBounds(const std::vector<double>& bounds);
  void Add(double v);
};

struct Point {
  Labels labels;
  ValueType value_type = ValueType::kInt64;
  int64_t int64_value = 0;
  double double_value = 0;
  std::string string_value;
  bool bool_value = false;
  Histogram histogram_value;
  int64_t start_timestamp_millis = 0;
  int64_t end_timestamp_millis = 0;
};

struct MetricDescriptor {
  std::string name;
  std::string description;
  std::vector<std::string> label_names;
  MetricKind kind = MetricKind::kCumulative;
  ValueType value_type = ValueType::kInt64;
};

struct PointSet {
  std::string metric_name;
  std::vector<std::unique_ptr<Point>> points;
};

struct CollectedMetrics {
  std::map<std::string, MetricDescriptor> descriptors;
  std::map<std::string, std::unique_ptr<PointSet>> point_sets;
};

int64_t NowMillis();

class MetricRegistry {
 public:
  static MetricRegistry* Default();

  void Define(const MetricDescriptor& d);
  void IncrementCounter(const std::string& name, int64_t delta, const Labels& labels = {});
  void SetGauge(const std::string& name, double value, const Labels& labels = {});
  void SetGaugeInt(const std::string& name, int64_t value, const Labels& labels = {});
  void SetGaugeString(const std::string& name, const std::string& value, const Labels& labels = {});
  void SetGaugeBool(const std::string& name, bool value, const Labels& labels = {});
  void Observe(const std::string& name, double value, const Labels& labels = {},
               const std::vector<double>& bounds = {});
  CollectedMetrics Collect() const;
  void Clear();

 private:
  struct Cell {
    Point point;
  };
  struct Metric {
    MetricDescriptor desc;
    std::vector<double> bounds;
    std::map<Labels, Cell> cells;
  };
  Metric& GetOrDefine(const std::string& name, MetricKind kind, ValueType vt);
  mutable std::mutex mu_;
  std::map<std::string, Metric> metrics_;
};

// ------------------------------------------------------------------ config --
class ExporterConfig {
 public:
  static ExporterConfig FromEnv();
  static const std::vector<std::string>& DefaultWhitelist();
  bool IsWhitelisted(const std::string& metric_name) const;
  std::string DebugString() const;

  bool enabled = false;
  std::string project_id;
  std::set<std::string> whitelist;
  int64_t interval_millis = 10 * 1000;
  std::string output_dir;
};

// --------------------------------------------------------------- converter --
struct Distribution {
  int64_t count = 0;
  double mean = 0;
  double sum_of_squared_deviation = 0;
  std::vector<double> bounds;
  std::vector<int64_t> bucket_counts;
};

struct TimeSeriesPoint {
  ValueType value_type = ValueType::kInt64;
  int64_t int64_value = 0;
  double double_value = 0;
  std::string string_value;
  bool bool_value = false;
  Distribution distribution;
  int64_t end_time_millis = 0;
};

struct TimeSeries {
  std::string metric_type;
  Labels metric_labels;
  std::string resource_type;
  std::vector<TimeSeriesPoint> points;
};

struct CreateTimeSeriesRequest {
  std::string name;  // "projects/<id>"
  std::vector<TimeSeries> time_series;
};

extern const char kMetricTypePrefix[];
extern const char kProjectNamePrefix[];
extern const char kDefaultResourceType[];

void ConvertDistribution(const Histogram& h, Distribution* out);
void ConvertPoint(const Point& p, TimeSeriesPoint* out);
void ConvertPointSet(const PointSet& ps, TimeSeries* out);
std::string TimeSeriesToJson(const TimeSeries& ts);
std::string DescriptorToJson(const MetricDescriptor& d, const std::string& metric_type);

// -------------------------------------------------------------------- sinks --
enum class Status { kOk, kAlreadyExists, kCancelled, kError };

class MetricSink {
 public:
  virtual ~MetricSink() = default;
  virtual Status CreateTimeSeries(const CreateTimeSeriesRequest& req) = 0;
  virtual Status CreateMetricDescriptor(const std::string& project_name, const MetricDescriptor& d,
                                        const std::string& metric_type) = 0;
};

class JsonlFileSink : public MetricSink {
 public:
  explicit JsonlFileSink(std::string dir);
  Status CreateTimeSeries(const CreateTimeSeriesRequest& req) override;
  Status CreateMetricDescriptor(const std::string& project_name, const MetricDescriptor& d,
                                const std::string& metric_type) override;

 private:
  std::string dir_;
  std::mutex mu_;
};

class PrometheusTextSink : public MetricSink {
 public:
  explicit PrometheusTextSink(std::string path);
  Status CreateTimeSeries(const CreateTimeSeriesRequest& req) override;
  Status CreateMetricDescriptor(const std::string&, const MetricDescriptor&, const std::string&) override {
    return Status::kOk;
  }

 private:
  std::string path_;
};

class RecordingSink : public MetricSink {
 public:
  Status CreateTimeSeries(const CreateTimeSeriesRequest& req) override;
  Status CreateMetricDescriptor(const std::string& project_name, const MetricDescriptor& d,
                                const std::string& metric_type) override;
  std::vector<CreateTimeSeriesRequest> series_requests;
  std::vector<std::string> descriptor_types;
  std::set<std::string> existing;  // descriptors reported as ALREADY_EXISTS
  std::mutex mu;
};

// ----------------------------------------------------------------- exporter --
class Exporter {
 public:
  Exporter(MetricRegistry* registry, std::shared_ptr<MetricSink> sink, ExporterConfig config);
  ~Exporter();
  // Idempotent: starts the background thread once (returns false if disabled).
  bool PeriodicallyExportMetrics();
  void ExportMetrics();
  void Stop();
  int64_t exports() const { return exports_.load(std::memory_order_acquire); }

  static bool ShouldExport(const PointSet& ps, const ExporterConfig& cfg);

 private:
  void ExportMetricDescriptors(const CollectedMetrics& m);
  MetricRegistry* registry_;
  std::shared_ptr<MetricSink> sink_;
  ExporterConfig config_;
  std::mutex mu_;
  std::mutex export_mu_;
  bool started_ = false;
  std::atomic<bool> stop_{false};
  std::thread thread_;
  std::set<std::string> exported_descriptors_;
  std::atomic<int64_t> exports_{0};  // read by other threads (found by the TSan CI variant)
};

}  // namespace monitoring
}  // namespace cloud_amd
