// Native input pipeline (pure C++ core, no Python): memory-mapped .npy sample arrays -> shuffled, rank-sharded
// batches gathered by a pool of C++ worker threads into caller-owned (pinned) slot
// buffers.  The Python side (cloud_amd/data/loader.py) copies a ready slot to the GPU
// on a copy stream and normalises it there (uint8 -> bf16 kernel), so host work
// never sits on the training stream.
//
// What the reference gets from tf.data (SURVEY.md 2.5 C4 "input sharding" and 2.7
// K9), done MI355X-side: one process per GPU, so every rank opens the same files
// and takes the rank-strided slice of a permutation that is identical on all ranks
// (seeded by (seed, epoch)); no communication.
//
// Lifecycle per epoch: start_epoch(e) builds the rank's index list and hands batch
// jobs to the workers as slots become free; next() returns the slot holding the
// next batch in order (blocking, GIL released); release(slot) recycles it.
#pragma once
#include <ctype.h>
#include <fcntl.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <numeric>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace ca_data {


// ----------------------------------------------------------------- .npy ----
struct NpyArray {
  std::string path;
  const uint8_t* data = nullptr;  // first element
  void* map = nullptr;
  size_t map_bytes = 0;
  std::string descr;
  size_t itemsize = 0;
  std::vector<long> shape;
  size_t row_bytes = 0;  // bytes of one sample (all dims but the first)
};

inline size_t itemsize_of(const std::string& d) {
  // '<u1', '|u1', '<f4', '<i8', '<f2', '|b1', ...
  if (d.size() < 3) throw std::runtime_error("npy: bad descr " + d);
  if (d[0] == '>') throw std::runtime_error("npy: big-endian arrays are not supported");
  return (size_t)std::stoul(d.substr(2));
}

inline std::string dict_value(const std::string& h, const std::string& key) {
  const size_t k = h.find("'" + key + "'");
  if (k == std::string::npos) throw std::runtime_error("npy: header lacks " + key);
  size_t p = h.find(':', k);
  if (p == std::string::npos) throw std::runtime_error("npy: malformed header");
  ++p;
  while (p < h.size() && h[p] == ' ') ++p;
  if (h[p] == '\'') {
    const size_t e = h.find('\'', p + 1);
    return h.substr(p + 1, e - p - 1);
  }
  if (h[p] == '(') {
    const size_t e = h.find(')', p);
    return h.substr(p, e - p + 1);
  }
  size_t e = p;
  while (e < h.size() && h[e] != ',' && h[e] != '}') ++e;
  return h.substr(p, e - p);
}

inline NpyArray open_npy(const std::string& path) {
  NpyArray a;
  a.path = path;
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("npy: cannot open " + path);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    ::close(fd);
    throw std::runtime_error("npy: cannot stat " + path);
  }
  a.map_bytes = (size_t)st.st_size;
  a.map = mmap(nullptr, a.map_bytes, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  if (a.map == MAP_FAILED) throw std::runtime_error("npy: mmap failed for " + path);
  const uint8_t* b = static_cast<const uint8_t*>(a.map);
  if (a.map_bytes < 10 || memcmp(b, "\x93NUMPY", 6) != 0) throw std::runtime_error("npy: bad magic in " + path);
  const int major = b[6];
  size_t hlen, hoff;
  if (major == 1) {
    hlen = b[8] | (b[9] << 8);
    hoff = 10;
  } else {
    hlen = b[8] | (b[9] << 8) | (b[10] << 16) | ((size_t)b[11] << 24);
    hoff = 12;
  }
  const std::string h(reinterpret_cast<const char*>(b + hoff), hlen);
  a.descr = dict_value(h, "descr");
  if (dict_value(h, "fortran_order").find("True") != std::string::npos)
    throw std::runtime_error("npy: fortran_order arrays are not supported");
  a.itemsize = itemsize_of(a.descr);
  const std::string sh = dict_value(h, "shape");
  for (size_t i = 1; i < sh.size();) {
    while (i < sh.size() && (sh[i] == ' ' || sh[i] == ',')) ++i;
    if (i >= sh.size() || sh[i] == ')') break;
    size_t j = i;
    while (j < sh.size() && isdigit((unsigned char)sh[j])) ++j;
    a.shape.push_back(std::stol(sh.substr(i, j - i)));
    i = j;
  }
  if (a.shape.empty()) throw std::runtime_error("npy: 0-d arrays are not sample arrays");
  a.row_bytes = a.itemsize;
  for (size_t d = 1; d < a.shape.size(); ++d) a.row_bytes *= (size_t)a.shape[d];
  a.data = b + hoff + hlen;
  if ((size_t)(a.data - b) + a.row_bytes * (size_t)a.shape[0] > a.map_bytes)
    throw std::runtime_error("npy: file shorter than its header says: " + path);
  madvise(a.map, a.map_bytes, MADV_RANDOM);
  return a;
}

// --------------------------------------------------------------- loader ----
enum SlotState { FREE = 0, FILLING = 1, READY = 2, HELD = 3 };

class Loader {
 public:
  Loader(const std::vector<std::string>& paths, long batch, bool shuffle, uint64_t seed, int rank, int world,
         bool drop_remainder, int threads, const std::vector<std::vector<uint64_t>>& slots)
      : batch_(batch), shuffle_(shuffle), seed_(seed), rank_(rank), world_(world), drop_(drop_remainder) {
    if (paths.empty()) throw std::invalid_argument("Loader: no arrays");
    if (batch <= 0 || world <= 0 || rank < 0 || rank >= world) throw std::invalid_argument("Loader: bad batch/rank");
    for (const auto& p : paths) arrays_.push_back(open_npy(p));
    n_ = arrays_[0].shape[0];
    for (const auto& a : arrays_)
      if (a.shape[0] != n_) throw std::invalid_argument("Loader: arrays differ in sample count");
    if (slots.empty()) throw std::invalid_argument("Loader: no slots");
    for (const auto& s : slots)
      if (s.size() != arrays_.size()) throw std::invalid_argument("Loader: one buffer per array per slot");
    slot_ptrs_ = slots;
    state_.assign(slots.size(), FREE);
    slot_batch_.assign(slots.size(), -1);
    slot_count_.assign(slots.size(), 0);
    for (int t = 0; t < std::max(1, threads); ++t) workers_.emplace_back([this] { work(); });
  }

  ~Loader() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_work_.notify_all();
    cv_ready_.notify_all();
    for (auto& w : workers_) w.join();
    for (auto& a : arrays_) munmap(a.map, a.map_bytes);
  }

  // Index list of this rank for `epoch`; returns the number of batches.
  long start_epoch(long epoch) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_ready_.wait(lk, [this] { return stop_ || in_flight_ == 0; });  // no worker touches the old list
    std::vector<long> perm(n_);
    std::iota(perm.begin(), perm.end(), 0L);
    if (shuffle_) {
      std::mt19937_64 rng(seed_ * 1000003ULL + (uint64_t)epoch);
      std::shuffle(perm.begin(), perm.end(), rng);
    }
    // equal share per rank (as DistributedSampler with drop_last): rank-strided
    const long per = n_ / world_;
    idx_.clear();
    idx_.reserve(per);
    for (long i = 0; i < per; ++i) idx_.push_back(perm[i * world_ + rank_]);
    nbatch_ = drop_ ? per / batch_ : (per + batch_ - 1) / batch_;
    next_job_ = 0;
    next_out_ = 0;
    for (size_t s = 0; s < state_.size(); ++s) {
      state_[s] = FREE;
      slot_batch_[s] = -1;
    }
    epoch_ = epoch;
    lk.unlock();
    cv_work_.notify_all();
    return nbatch_;
  }

  // Blocks until the next batch (in order) is ready; returns (slot, samples) or (-1, 0) at epoch end.
  std::pair<int, long> next() {
    std::unique_lock<std::mutex> lk(mu_);
    if (next_out_ >= nbatch_) return {-1, 0};
    const long want = next_out_;
    int slot = -1;
    cv_ready_.wait(lk, [&] {
      if (stop_ || !error_.empty()) return true;
      for (size_t s = 0; s < state_.size(); ++s)
        if (state_[s] == READY && slot_batch_[s] == want) {
          slot = (int)s;
          return true;
        }
      return false;
    });
    if (!error_.empty()) throw std::runtime_error(error_);
    if (slot < 0) return {-1, 0};
    state_[slot] = HELD;
    ++next_out_;
    return {slot, slot_count_[slot]};
  }

  void release(int slot) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (slot < 0 || slot >= (int)state_.size() || state_[slot] != HELD)
        throw std::invalid_argument("Loader.release: slot not held");
      state_[slot] = FREE;
      slot_batch_[slot] = -1;
    }
    cv_work_.notify_all();
  }

  long num_samples() const { return n_; }
  long epoch() const { return epoch_; }
  const std::vector<NpyArray>& arrays() const { return arrays_; }

 private:
  void work() {
    for (;;) {
      int slot = -1;
      long b = -1;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_work_.wait(lk, [&] {
          if (stop_) return true;
          if (next_job_ >= nbatch_) return false;
          // never run more than #slots batches ahead of the consumer
          if (next_job_ >= next_out_ + (long)state_.size()) return false;
          for (size_t s = 0; s < state_.size(); ++s)
            if (state_[s] == FREE) {
              slot = (int)s;
              return true;
            }
          return false;
        });
        if (stop_) return;
        b = next_job_++;
        state_[slot] = FILLING;
        slot_batch_[slot] = b;
        ++in_flight_;
      }
      const long lo = b * batch_;
      const long hi = std::min<long>(lo + batch_, (long)idx_.size());
      try {
        for (size_t a = 0; a < arrays_.size(); ++a) {
          const NpyArray& arr = arrays_[a];
          uint8_t* dst = reinterpret_cast<uint8_t*>(slot_ptrs_[slot][a]);
          for (long i = lo; i < hi; ++i)
            memcpy(dst + (size_t)(i - lo) * arr.row_bytes, arr.data + (size_t)idx_[i] * arr.row_bytes, arr.row_bytes);
        }
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(mu_);
        error_ = e.what();
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        slot_count_[slot] = hi - lo;
        state_[slot] = READY;
        --in_flight_;
      }
      cv_ready_.notify_all();
    }
  }

  std::vector<NpyArray> arrays_;
  long n_ = 0, batch_;
  bool shuffle_;
  uint64_t seed_;
  int rank_, world_;
  bool drop_;
  std::vector<std::vector<uint64_t>> slot_ptrs_;
  std::vector<int> state_;
  std::vector<long> slot_batch_, slot_count_;
  std::vector<long> idx_;
  long nbatch_ = 0, next_job_ = 0, next_out_ = 0, epoch_ = -1;
  int in_flight_ = 0;
  bool stop_ = false;
  std::string error_;
  std::mutex mu_;
  std::condition_variable cv_work_, cv_ready_;
  std::vector<std::thread> workers_;
};

}  // namespace ca_data
