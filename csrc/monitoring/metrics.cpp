// Implementation of the cloud_amd metrics registry / converter / sinks / exporter.
// See metrics.h for the mapping onto reference src/cpp/monitoring/*.
#include "metrics.h"

#include <fcntl.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <limits>
#include <sstream>
#include <sys/stat.h>

namespace cloud_amd {
namespace monitoring {

const char kMetricTypePrefix[] = "custom.cloud_amd";
const char kProjectNamePrefix[] = "projects/";
const char kDefaultResourceType[] = "global";

int64_t NowMillis() {
  using namespace std::chrono;
  return duration_cast<milliseconds>(system_clock::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------- Histogram --
Histogram Histogram::WithBounds(const std::vector<double>& bounds) {
  Histogram h;
  h.bucket_limits = bounds;
  h.bucket_limits.push_back(std::numeric_limits<double>::max());
  h.bucket_counts.assign(h.bucket_limits.size(), 0.0);
  return h;
}

void Histogram::Add(double v) {
  size_t i = 0;
  while (i + 1 < bucket_limits.size() && v >= bucket_limits[i]) ++i;
  if (bucket_counts.empty()) {
    bucket_limits.push_back(std::numeric_limits<double>::max());
    bucket_counts.push_back(0);
  }
  bucket_counts[i] += 1;
  if (num == 0) {
    min = max = v;
  } else {
    min = std::min(min, v);
    max = std::max(max, v);
  }
  num += 1;
  sum += v;
  sum_squares += v * v;
}

// ----------------------------------------------------------------- Registry --
MetricRegistry* MetricRegistry::Default() {
  static MetricRegistry* r = new MetricRegistry();
  return r;
}

void MetricRegistry::Define(const MetricDescriptor& d) {
  std::lock_guard<std::mutex> l(mu_);
  auto& m = metrics_[d.name];
  m.desc = d;
}

MetricRegistry::Metric& MetricRegistry::GetOrDefine(const std::string& name, MetricKind kind, ValueType vt) {
  auto it = metrics_.find(name);
  if (it == metrics_.end()) {
    Metric m;
    m.desc.name = name;
    m.desc.kind = kind;
    m.desc.value_type = vt;
    it = metrics_.emplace(name, std::move(m)).first;
  }
  return it->second;
}

void MetricRegistry::IncrementCounter(const std::string& name, int64_t delta, const Labels& labels) {
  std::lock_guard<std::mutex> l(mu_);
  auto& m = GetOrDefine(name, MetricKind::kCumulative, ValueType::kInt64);
  auto& c = m.cells[labels];
  if (c.point.start_timestamp_millis == 0) c.point.start_timestamp_millis = NowMillis();
  c.point.labels = labels;
  c.point.value_type = ValueType::kInt64;
  c.point.int64_value += delta;
  c.point.end_timestamp_millis = NowMillis();
}

#define CA_GAUGE_SET(FIELD, VT)                                          \
  std::lock_guard<std::mutex> l(mu_);                                    \
  auto& m = GetOrDefine(name, MetricKind::kGauge, VT);                   \
  auto& c = m.cells[labels];                                             \
  c.point.labels = labels;                                               \
  c.point.value_type = VT;                                               \
  c.point.FIELD = value;                                                 \
  c.point.end_timestamp_millis = NowMillis();

void MetricRegistry::SetGauge(const std::string& name, double value, const Labels& labels) {
  CA_GAUGE_SET(double_value, ValueType::kDouble)
}
void MetricRegistry::SetGaugeInt(const std::string& name, int64_t value, const Labels& labels) {
  CA_GAUGE_SET(int64_value, ValueType::kInt64)
}
void MetricRegistry::SetGaugeString(const std::string& name, const std::string& value, const Labels& labels) {
  CA_GAUGE_SET(string_value, ValueType::kString)
}
void MetricRegistry::SetGaugeBool(const std::string& name, bool value, const Labels& labels) {
  CA_GAUGE_SET(bool_value, ValueType::kBool)
}
#undef CA_GAUGE_SET

void MetricRegistry::Observe(const std::string& name, double value, const Labels& labels,
                             const std::vector<double>& bounds) {
  std::lock_guard<std::mutex> l(mu_);
  auto& m = GetOrDefine(name, MetricKind::kCumulative, ValueType::kHistogram);
  if (m.bounds.empty()) {
    if (!bounds.empty()) {
      m.bounds = bounds;
    } else {  // exponential default: 1e-3 .. ~1e6 (ms-friendly)
      for (double b = 1e-3; b < 1e7; b *= 2) m.bounds.push_back(b);
    }
  }
  auto it = m.cells.find(labels);
  if (it == m.cells.end()) {
    Cell c;
    c.point.labels = labels;
    c.point.value_type = ValueType::kHistogram;
    c.point.histogram_value = Histogram::WithBounds(m.bounds);
    c.point.start_timestamp_millis = NowMillis();
    it = m.cells.emplace(labels, std::move(c)).first;
  }
  it->second.point.histogram_value.Add(value);
  it->second.point.end_timestamp_millis = NowMillis();
}

CollectedMetrics MetricRegistry::Collect() const {
  std::lock_guard<std::mutex> l(mu_);
  CollectedMetrics out;
  for (const auto& kv : metrics_) {
    out.descriptors[kv.first] = kv.second.desc;
    auto ps = std::make_unique<PointSet>();
    ps->metric_name = kv.first;
    for (const auto& cell : kv.second.cells) ps->points.push_back(std::make_unique<Point>(cell.second.point));
    out.point_sets[kv.first] = std::move(ps);
  }
  return out;
}

void MetricRegistry::Clear() {
  std::lock_guard<std::mutex> l(mu_);
  metrics_.clear();
}

// ------------------------------------------------------------------- Config --
const std::vector<std::string>& ExporterConfig::DefaultWhitelist() {
  static const std::vector<std::string> kList = {
      "/cloud_amd/train/step_time_ms",       "/cloud_amd/train/images_per_sec",
      "/cloud_amd/train/first_step_latency_s", "/cloud_amd/comm/allreduce_ms",
      "/cloud_amd/comm/exposed_ms",
      "/cloud_amd/data/getnext_duration_us", "/cloud_amd/data/getnext_period_us",
      "/cloud_amd/data/bytes_fetched",       "/cloud_amd/kernel/time_us",
      "/cloud_amd/tuner/trials",             "/cloud_amd/launcher/jobs",
  };
  return kList;
}

static bool EnvBool(const char* name, bool dflt) {
  const char* v = std::getenv(name);
  if (!v) return dflt;
  std::string s(v);
  for (auto& ch : s) ch = (char)std::tolower(ch);
  return s == "1" || s == "true" || s == "yes";
}

ExporterConfig ExporterConfig::FromEnv() {
  ExporterConfig c;
  c.enabled = EnvBool("CLOUD_AMD_MONITORING_EXPORTER_ENABLED", false);
  if (const char* p = std::getenv("CLOUD_AMD_MONITORING_PROJECT_ID")) c.project_id = p;
  if (c.project_id.empty()) c.project_id = "local";
  const char* wl = std::getenv("CLOUD_AMD_MONITORING_METRICS_WHITELIST");
  if (wl && *wl) {
    std::stringstream ss(wl);
    std::string item;
    while (std::getline(ss, item, ',')) {
      if (!item.empty()) c.whitelist.insert(item);
    }
  } else {
    c.whitelist.insert(DefaultWhitelist().begin(), DefaultWhitelist().end());
  }
  if (const char* iv = std::getenv("CLOUD_AMD_MONITORING_INTERVAL_S")) {
    c.interval_millis = (int64_t)(std::atof(iv) * 1000.0);
    if (c.interval_millis < 10) c.interval_millis = 10;
  }
  if (const char* d = std::getenv("CLOUD_AMD_MONITORING_DIR")) c.output_dir = d;
  return c;
}

bool ExporterConfig::IsWhitelisted(const std::string& metric_name) const {
  return whitelist.count(metric_name) > 0;
}

std::string ExporterConfig::DebugString() const {
  std::ostringstream os;
  os << "ExporterConfig{enabled=" << enabled << ", project_id=" << project_id << ", interval_ms=" << interval_millis
     << ", whitelist=[";
  bool first = true;
  for (const auto& w : whitelist) {
    os << (first ? "" : ", ") << w;
    first = false;
  }
  os << "]}";
  return os.str();
}

// ---------------------------------------------------------------- Converter --
void ConvertDistribution(const Histogram& h, Distribution* d) {
  d->count = (int64_t)h.num;
  if (h.num != 0.0) {
    d->mean = h.sum / h.num;
    d->sum_of_squared_deviation = (h.sum_squares * h.num - h.sum * h.sum) / h.num;
  } else {
    d->mean = 0.0;
    d->sum_of_squared_deviation = 0.0;
  }
  d->bounds.clear();
  for (size_t i = 0; i + 1 < h.bucket_limits.size(); ++i) d->bounds.push_back(h.bucket_limits[i]);
  d->bucket_counts.clear();
  for (double c : h.bucket_counts) d->bucket_counts.push_back((int64_t)c);
}

void ConvertPoint(const Point& p, TimeSeriesPoint* out) {
  out->value_type = p.value_type;
  switch (p.value_type) {
    case ValueType::kInt64: out->int64_value = p.int64_value; break;
    case ValueType::kDouble: out->double_value = p.double_value; break;
    case ValueType::kString: out->string_value = p.string_value; break;
    case ValueType::kBool: out->bool_value = p.bool_value; break;
    case ValueType::kHistogram: ConvertDistribution(p.histogram_value, &out->distribution); break;
  }
  out->end_time_millis = p.end_timestamp_millis;
}

void ConvertPointSet(const PointSet& ps, TimeSeries* ts) {
  ts->metric_type = std::string(kMetricTypePrefix) + ps.metric_name;
  ts->resource_type = kDefaultResourceType;
  if (!ps.points.empty()) {  // first point only (reference keeps the first point)
    ts->metric_labels = ps.points.front()->labels;
    TimeSeriesPoint tp;
    ConvertPoint(*ps.points.front(), &tp);
    ts->points.push_back(tp);
  }
}

static std::string JsonEscape(const std::string& s) {
  std::string o;
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      default: o += c;
    }
  }
  return o;
}

static std::string Num(double v) {
  if (!std::isfinite(v)) return v > 0 ? "1e308" : (v < 0 ? "-1e308" : "0");
  std::ostringstream os;
  os.precision(17);
  os << v;
  return os.str();
}

std::string TimeSeriesToJson(const TimeSeries& ts) {
  std::ostringstream os;
  os << "{\"metric\":{\"type\":\"" << JsonEscape(ts.metric_type) << "\",\"labels\":{";
  bool first = true;
  for (const auto& kv : ts.metric_labels) {
    os << (first ? "" : ",") << "\"" << JsonEscape(kv.first) << "\":\"" << JsonEscape(kv.second) << "\"";
    first = false;
  }
  os << "}},\"resource\":{\"type\":\"" << ts.resource_type << "\"},\"points\":[";
  for (size_t i = 0; i < ts.points.size(); ++i) {
    const auto& p = ts.points[i];
    os << (i ? "," : "") << "{\"interval\":{\"endTimeMillis\":" << p.end_time_millis << "},\"value\":{";
    switch (p.value_type) {
      case ValueType::kInt64: os << "\"int64Value\":" << p.int64_value; break;
      case ValueType::kDouble: os << "\"doubleValue\":" << Num(p.double_value); break;
      case ValueType::kString: os << "\"stringValue\":\"" << JsonEscape(p.string_value) << "\""; break;
      case ValueType::kBool: os << "\"boolValue\":" << (p.bool_value ? "true" : "false"); break;
      case ValueType::kHistogram: {
        const auto& d = p.distribution;
        os << "\"distributionValue\":{\"count\":" << d.count << ",\"mean\":" << Num(d.mean)
           << ",\"sumOfSquaredDeviation\":" << Num(d.sum_of_squared_deviation)
           << ",\"bucketOptions\":{\"explicitBuckets\":{\"bounds\":[";
        for (size_t j = 0; j < d.bounds.size(); ++j) os << (j ? "," : "") << Num(d.bounds[j]);
        os << "]}},\"bucketCounts\":[";
        for (size_t j = 0; j < d.bucket_counts.size(); ++j) os << (j ? "," : "") << d.bucket_counts[j];
        os << "]}";
        break;
      }
    }
    os << "}}";
  }
  os << "]}";
  return os.str();
}

static const char* KindName(MetricKind k) { return k == MetricKind::kGauge ? "GAUGE" : "CUMULATIVE"; }
static const char* TypeName(ValueType t) {
  switch (t) {
    case ValueType::kInt64: return "INT64";
    case ValueType::kDouble: return "DOUBLE";
    case ValueType::kString: return "STRING";
    case ValueType::kBool: return "BOOL";
    case ValueType::kHistogram: return "DISTRIBUTION";
  }
  return "VALUE_TYPE_UNSPECIFIED";
}

std::string DescriptorToJson(const MetricDescriptor& d, const std::string& metric_type) {
  std::ostringstream os;
  os << "{\"type\":\"" << JsonEscape(metric_type) << "\",\"description\":\"" << JsonEscape(d.description)
     << "\",\"metricKind\":\"" << KindName(d.kind) << "\",\"valueType\":\"" << TypeName(d.value_type)
     << "\",\"labels\":[";
  for (size_t i = 0; i < d.label_names.size(); ++i)
    os << (i ? "," : "") << "{\"key\":\"" << JsonEscape(d.label_names[i]) << "\",\"valueType\":\"STRING\"}";
  os << "]}";
  return os.str();
}

// -------------------------------------------------------------------- Sinks --
static void MakeDirs(const std::string& dir) {
  std::string cur;
  for (size_t i = 0; i < dir.size(); ++i) {
    cur += dir[i];
    if (dir[i] == '/' || i + 1 == dir.size()) mkdir(cur.c_str(), 0755);
  }
}

JsonlFileSink::JsonlFileSink(std::string dir) : dir_(std::move(dir)) { MakeDirs(dir_); }

// Every rank of a job appends to the same file: one export is formatted into one
// buffer and written with a single write(2) on an O_APPEND descriptor, so lines of
// different processes never interleave.
static Status AppendAll(const std::string& path, const std::string& text) {
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
  if (fd < 0) return Status::kError;
  size_t off = 0;
  while (off < text.size()) {
    const ssize_t w = ::write(fd, text.data() + off, text.size() - off);
    if (w <= 0) {
      ::close(fd);
      return Status::kError;
    }
    off += (size_t)w;
  }
  ::close(fd);
  return Status::kOk;
}

Status JsonlFileSink::CreateTimeSeries(const CreateTimeSeriesRequest& req) {
  if (req.time_series.empty()) return Status::kCancelled;
  std::lock_guard<std::mutex> l(mu_);
  const int64_t now = NowMillis();
  std::ostringstream os;
  for (const auto& ts : req.time_series)
    os << "{\"name\":\"" << req.name << "\",\"exportTimeMillis\":" << now << ",\"timeSeries\":" << TimeSeriesToJson(ts)
       << "}\n";
  return AppendAll(dir_ + "/metrics.jsonl", os.str());
}

Status JsonlFileSink::CreateMetricDescriptor(const std::string& project_name, const MetricDescriptor& d,
                                             const std::string& metric_type) {
  std::lock_guard<std::mutex> l(mu_);
  return AppendAll(dir_ + "/descriptors.jsonl",
                   "{\"name\":\"" + project_name + "\",\"metricDescriptor\":" + DescriptorToJson(d, metric_type) + "}\n");
}

PrometheusTextSink::PrometheusTextSink(std::string path) : path_(std::move(path)) {}

static std::string PromName(const std::string& metric_type) {
  std::string o;
  for (char c : metric_type) o += (std::isalnum((unsigned char)c) ? c : '_');
  return o;
}

Status PrometheusTextSink::CreateTimeSeries(const CreateTimeSeriesRequest& req) {
  if (req.time_series.empty()) return Status::kCancelled;
  std::ostringstream os;
  for (const auto& ts : req.time_series) {
    if (ts.points.empty()) continue;
    std::string name = PromName(ts.metric_type);
    std::string lbl;
    for (const auto& kv : ts.metric_labels) lbl += (lbl.empty() ? "" : ",") + kv.first + "=\"" + kv.second + "\"";
    const auto& p = ts.points.front();
    auto with = [&](const std::string& extra) {
      std::string all = lbl;
      if (!extra.empty()) all += (all.empty() ? "" : ",") + extra;
      return all.empty() ? std::string() : "{" + all + "}";
    };
    switch (p.value_type) {
      case ValueType::kInt64: os << name << with("") << " " << p.int64_value << "\n"; break;
      case ValueType::kDouble: os << name << with("") << " " << Num(p.double_value) << "\n"; break;
      case ValueType::kBool: os << name << with("") << " " << (p.bool_value ? 1 : 0) << "\n"; break;
      case ValueType::kString: os << name << with("value=\"" + p.string_value + "\"") << " 1\n"; break;
      case ValueType::kHistogram: {
        int64_t cum = 0;
        const auto& d = p.distribution;
        for (size_t i = 0; i < d.bucket_counts.size(); ++i) {
          cum += d.bucket_counts[i];
          std::string le = i < d.bounds.size() ? Num(d.bounds[i]) : "+Inf";
          os << name << "_bucket" << with("le=\"" + le + "\"") << " " << cum << "\n";
        }
        os << name << "_count" << with("") << " " << d.count << "\n";
        os << name << "_sum" << with("") << " " << Num(d.mean * (double)d.count) << "\n";
        break;
      }
    }
  }
  const std::string tmp = path_ + ".tmp";
  {
    std::ofstream f(tmp, std::ios::trunc);
    if (!f) return Status::kError;
    f << os.str();
  }
  return std::rename(tmp.c_str(), path_.c_str()) == 0 ? Status::kOk : Status::kError;
}

Status RecordingSink::CreateTimeSeries(const CreateTimeSeriesRequest& req) {
  if (req.time_series.empty()) return Status::kCancelled;
  std::lock_guard<std::mutex> l(mu);
  series_requests.push_back(req);
  return Status::kOk;
}

Status RecordingSink::CreateMetricDescriptor(const std::string&, const MetricDescriptor&, const std::string& type) {
  std::lock_guard<std::mutex> l(mu);
  descriptor_types.push_back(type);
  return existing.count(type) ? Status::kAlreadyExists : Status::kOk;
}

// ----------------------------------------------------------------- Exporter --
Exporter::Exporter(MetricRegistry* registry, std::shared_ptr<MetricSink> sink, ExporterConfig config)
    : registry_(registry), sink_(std::move(sink)), config_(std::move(config)) {}

Exporter::~Exporter() { Stop(); }

bool Exporter::ShouldExport(const PointSet& ps, const ExporterConfig& cfg) {
  if (!cfg.IsWhitelisted(ps.metric_name)) return false;
  size_t non_empty = 0;
  for (const auto& p : ps.points) {
    switch (p->value_type) {
      case ValueType::kInt64: non_empty += p->int64_value != 0; break;
      case ValueType::kHistogram: non_empty += p->histogram_value.num > 0; break;
      case ValueType::kDouble: non_empty += p->double_value != 0.0; break;
      default: break;  // other value types are not exported (as in the reference)
    }
  }
  return non_empty > 0;
}

bool Exporter::PeriodicallyExportMetrics() {
  std::lock_guard<std::mutex> l(mu_);
  if (!config_.enabled) return false;
  if (started_) return true;
  started_ = true;
  stop_.store(false);
  // Sleep in <= 10 ms slices on an atomic flag (no condition variable: Stop()
  // returns promptly and the thread is clean under ThreadSanitizer).
  thread_ = std::thread([this] {
    const auto interval = std::chrono::milliseconds(config_.interval_millis);
    while (!stop_.load(std::memory_order_acquire)) {
      const auto deadline = std::chrono::steady_clock::now() + interval;
      while (!stop_.load(std::memory_order_acquire) && std::chrono::steady_clock::now() < deadline)
        std::this_thread::sleep_for(std::min<std::chrono::steady_clock::duration>(
            std::chrono::milliseconds(10), deadline - std::chrono::steady_clock::now()));
      if (stop_.load(std::memory_order_acquire)) break;
      ExportMetrics();
    }
  });
  return true;
}

void Exporter::ExportMetricDescriptors(const CollectedMetrics& m) {
  for (const auto& kv : m.point_sets) {
    const std::string& name = kv.first;
    if (exported_descriptors_.count(name)) continue;
    auto it = m.descriptors.find(name);
    if (it == m.descriptors.end()) continue;
    const Status s = sink_->CreateMetricDescriptor(std::string(kProjectNamePrefix) + config_.project_id, it->second,
                                                   std::string(kMetricTypePrefix) + name);
    if (s == Status::kOk || s == Status::kAlreadyExists) exported_descriptors_.insert(name);
  }
}

void Exporter::ExportMetrics() {
  std::lock_guard<std::mutex> guard(export_mu_);
  CollectedMetrics all = registry_->Collect();
  CollectedMetrics solid;
  for (auto& kv : all.point_sets) {
    if (ShouldExport(*kv.second, config_)) {
      solid.descriptors[kv.first] = all.descriptors[kv.first];
      solid.point_sets.emplace(kv.first, std::move(kv.second));
    }
  }
  if (solid.point_sets.empty()) return;
  ExportMetricDescriptors(solid);
  CreateTimeSeriesRequest req;
  req.name = std::string(kProjectNamePrefix) + config_.project_id;
  for (const auto& kv : solid.point_sets) {
    TimeSeries ts;
    ConvertPointSet(*kv.second, &ts);
    req.time_series.push_back(ts);
  }
  if (sink_->CreateTimeSeries(req) != Status::kOk) {
    std::fprintf(stderr, "[cloud_amd.monitoring] failed to export %zu time series\n", req.time_series.size());
  }
  exports_.fetch_add(1, std::memory_order_release);
}

void Exporter::Stop() {
  std::lock_guard<std::mutex> l(mu_);
  if (!started_) return;
  stop_.store(true, std::memory_order_release);
  if (thread_.joinable()) thread_.join();
  started_ = false;
}

}  // namespace monitoring
}  // namespace cloud_amd
