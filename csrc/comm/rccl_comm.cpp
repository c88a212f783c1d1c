// Native RCCL communicator for cloud_amd's data-parallel engine (C1/C2 in
// SURVEY.md 2.5): one communicator per process (one process per MI355X),
// collectives enqueued on a dedicated high-priority HIP "comm" stream that
// waits on an event recorded on the compute stream -- so a gradient bucket's
// all-reduce starts as soon as the backward kernels that produced it retire
// and runs concurrently with the rest of the backward.  join() makes the
// compute stream wait for everything issued so far (before the optimizer).
//
// Bootstrap: rank 0 calls unique_id() and publishes the 128-byte id through the
// rendezvous store (cloud_amd/parallel/comm.py); every rank then constructs
// Comm(nranks, rank, id, device, timeout_s) -> ncclCommInitRankConfig in NON-BLOCKING mode,
// polled with ncclCommGetAsyncError until it settles or the deadline passes; past the
// deadline the half-built communicator is aborted (ncclCommAbort) and the constructor
// raises TimeoutError -- a peer that hangs before joining (rather than exiting) no longer
// stalls every rank until the launcher's job timeout.  In non-blocking mode any call may
// return ncclInProgress; settle() polls it to completion with the GIL released.
//
// Lifetime: every use of comm_ happens under mu_, taken only with the GIL released (so a
// thread waiting for mu_ never holds the GIL another thread needs to finish).  abort()
// (the Python watchdog's thread) first raises abort_req_: a settle() or finalize loop in
// flight sees it, aborts the communicator itself and raises, and only then does abort()
// get mu_ -- comm_ is never freed under a poller.  settle() and the finalize loop also
// have a deadline (timeout_s): a peer that keeps a call ncclInProgress forever ends in
// ncclCommAbort + an exception instead of a spin.  async_error() only try-locks: while a
// call is in flight it answers "healthy" (that call polls the same state itself).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

namespace py = pybind11;

namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

ncclDataType_t dtype_of(int code) {
  switch (code) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclInt32;
    case 4: return ncclInt64;
    case 5: return ncclUint8;
  }
  throw std::invalid_argument("unsupported dtype code");
}

ncclRedOp_t op_of(int code) {
  switch (code) {
    case 0: return ncclSum;
    case 1: return ncclMax;
    case 2: return ncclMin;
    case 3: return ncclAvg;
  }
  throw std::invalid_argument("unsupported reduce op");
}

hipStream_t S(uint64_t s) { return reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(s)); }
void* P(uint64_t p) { return reinterpret_cast<void*>(static_cast<uintptr_t>(p)); }

struct InitTimeout : std::runtime_error {
  using std::runtime_error::runtime_error;
};

double since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

class Comm {
 public:
  Comm(int nranks, int rank, py::bytes uid, int device, double timeout_s)
      : timeout_s_(timeout_s), nranks_(nranks), rank_(rank), device_(device) {
    std::string u = uid;
    if (u.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("unique id must be 128 bytes");
    ncclUniqueId id;
    memcpy(&id, u.data(), sizeof(id));
    hip_check(hipSetDevice(device), "hipSetDevice");
    int lo = 0, hi = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
    hip_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "hipStreamCreateWithPriority");
    hip_check(hipEventCreateWithFlags(&ready_, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&done_, hipEventDisableTiming), "hipEventCreate");
    auto t0 = std::chrono::steady_clock::now();
    ncclResult_t state = ncclSuccess;
    {
      py::gil_scoped_release nogil;  // init completes only when every rank joined
      ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
      cfg.blocking = 0;
      ncclResult_t r = ncclCommInitRankConfig(&comm_, nranks, id, rank, &cfg);
      if (r != ncclSuccess && r != ncclInProgress) {
        comm_ = nullptr;
        destroy_locked();
        nccl_check(r, "ncclCommInitRankConfig");
      }
      state = r;
      while (state == ncclInProgress) {
        if (ncclCommGetAsyncError(comm_, &state) != ncclSuccess) break;
        if (state != ncclInProgress) break;
        double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (timeout_s > 0 && el > timeout_s) {
          ncclCommAbort(comm_);  // unblocks the init threads; frees the partial communicator
          comm_ = nullptr;
          break;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
      }
    }
    init_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!comm_) {
      destroy_locked();
      throw InitTimeout("ncclCommInitRankConfig: rank " + std::to_string(rank) + " of " + std::to_string(nranks) +
                        " not joined by all peers within " + std::to_string(timeout_s) + " s (aborted)");
    }
    if (state != ncclSuccess) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
      destroy_locked();
      nccl_check(state, "ncclCommInitRankConfig (async)");
    }
  }

  ~Comm() {
    try {
      destroy();
    } catch (...) {
    }
  }

  void destroy() {
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> g(mu_);
    destroy_locked();
  }

  void abort() {
    abort_req_.store(true);
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> g(mu_);  // a poller in flight aborts and releases first
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }

  void all_reduce(uint64_t buf, size_t count, int dtype, int op, uint64_t compute) {
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> g(mu_);
    after_locked(compute);
    settle(ncclAllReduce(P(buf), P(buf), count, dtype_of(dtype), op_of(op), comm_, stream_), "ncclAllReduce");
  }

  void broadcast(uint64_t buf, size_t count, int dtype, int root, uint64_t compute) {
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> g(mu_);
    after_locked(compute);
    settle(ncclBroadcast(P(buf), P(buf), count, dtype_of(dtype), root, comm_, stream_), "ncclBroadcast");
  }

  void reduce_scatter(uint64_t send, uint64_t recv, size_t recvcount, int dtype, int op, uint64_t compute) {
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> g(mu_);
    after_locked(compute);
    settle(ncclReduceScatter(P(send), P(recv), recvcount, dtype_of(dtype), op_of(op), comm_, stream_),
           "ncclReduceScatter");
  }

  void all_gather(uint64_t send, uint64_t recv, size_t sendcount, int dtype, uint64_t compute) {
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> g(mu_);
    after_locked(compute);
    settle(ncclAllGather(P(send), P(recv), sendcount, dtype_of(dtype), comm_, stream_), "ncclAllGather");
  }

  // compute stream waits for every collective issued so far
  void join(uint64_t compute) {
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> g(mu_);
    live();
    hip_check(hipEventRecord(done_, stream_), "hipEventRecord");
    hip_check(hipStreamWaitEvent(S(compute), done_, 0), "hipStreamWaitEvent");
  }

  // polls instead of blocking in hipStreamSynchronize, so an abort ends the wait
  void synchronize() {
    py::gil_scoped_release nogil;
    hipStream_t s;
    {
      std::lock_guard<std::mutex> g(mu_);
      live();
      s = stream_;
    }
    for (;;) {
      hipError_t e = hipStreamQuery(s);
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady) hip_check(e, "hipStreamQuery");
      if (abort_req_.load()) throw std::runtime_error("synchronize: communicator aborted");
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }

  // 0 = healthy (or a call in flight); otherwise the ncclResult_t of an asynchronous failure
  int async_error() {
    py::gil_scoped_release nogil;
    std::unique_lock<std::mutex> g(mu_, std::try_to_lock);
    if (!g.owns_lock()) return 0;
    if (!comm_) return -1;
    ncclResult_t r = ncclSuccess;
    nccl_check(ncclCommGetAsyncError(comm_, &r), "ncclCommGetAsyncError");
    return (int)r;
  }

  uint64_t stream() const { return reinterpret_cast<uintptr_t>(stream_); }
  double init_seconds() const { return init_s_; }
  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  int device() const { return device_; }

 private:
  void live() const {
    if (!comm_) throw std::runtime_error("communicator destroyed or aborted");
  }

  // comm stream waits for the work already queued on the compute stream (mu_ held)
  void after_locked(uint64_t compute) {
    live();
    hip_check(hipEventRecord(ready_, S(compute)), "hipEventRecord");
    hip_check(hipStreamWaitEvent(stream_, ready_, 0), "hipStreamWaitEvent");
  }

  void abort_locked() {
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }

  // a non-blocking communicator may answer ncclInProgress: the call is enqueued once its
  // state settles.  Ends on success, an error, abort() or the deadline (mu_ held).
  void settle(ncclResult_t r, const char* what) {
    auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress) {
      if (abort_req_.load()) {
        abort_locked();
        throw std::runtime_error(std::string(what) + ": communicator aborted");
      }
      if (timeout_s_ > 0 && since(t0) > timeout_s_) {
        abort_locked();
        throw std::runtime_error(std::string(what) + ": still in progress after " + std::to_string(timeout_s_) +
                                 " s (communicator aborted)");
      }
      std::this_thread::yield();
      if (ncclCommGetAsyncError(comm_, &r) != ncclSuccess) break;
    }
    nccl_check(r, what);
  }

  // finalize (flush) and destroy; abort instead when an abort was asked for or the
  // finalize does not settle within the deadline (mu_ held, or not shared yet)
  void destroy_locked() {
    if (comm_) {
      if (abort_req_.load()) {
        abort_locked();
      } else {
        hipStreamSynchronize(stream_);
        ncclResult_t st = ncclCommFinalize(comm_);
        auto t0 = std::chrono::steady_clock::now();
        while (st == ncclInProgress) {
          if (abort_req_.load() || (timeout_s_ > 0 && since(t0) > timeout_s_)) {
            abort_locked();
            break;
          }
          std::this_thread::yield();
          if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) break;
        }
        if (comm_) {
          ncclCommDestroy(comm_);
          comm_ = nullptr;
        }
      }
    }
    if (stream_) {
      hipEventDestroy(ready_);
      hipEventDestroy(done_);
      hipStreamDestroy(stream_);
      stream_ = nullptr;
    }
  }

  std::mutex mu_;
  std::atomic<bool> abort_req_{false};
  double timeout_s_;
  double init_s_ = 0.0;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  hipEvent_t ready_ = nullptr, done_ = nullptr;
  int nranks_, rank_, device_;
};

}  // namespace

PYBIND11_MODULE(_comm, m) {
  m.doc() = "cloud_amd native RCCL communicator (collectives on a side HIP stream)";
  m.def("unique_id", []() {
    ncclUniqueId id;
    nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
  });
  m.def("version", []() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });
  py::register_exception<InitTimeout>(m, "InitTimeout", PyExc_TimeoutError);
  py::class_<Comm>(m, "Comm")
      .def(py::init<int, int, py::bytes, int, double>(), py::arg("nranks"), py::arg("rank"), py::arg("uid"),
           py::arg("device"), py::arg("timeout_s") = 600.0)
      .def("all_reduce", &Comm::all_reduce)
      .def("broadcast", &Comm::broadcast)
      .def("reduce_scatter", &Comm::reduce_scatter)
      .def("all_gather", &Comm::all_gather)
      .def("join", &Comm::join)
      .def("synchronize", &Comm::synchronize)
      .def("async_error", &Comm::async_error)
      .def("abort", &Comm::abort)
      .def("destroy", &Comm::destroy)
      .def_property_readonly("stream", &Comm::stream)
      .def_property_readonly("init_seconds", &Comm::init_seconds)
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("nranks", &Comm::nranks)
      .def_property_readonly("device", &Comm::device);
}
