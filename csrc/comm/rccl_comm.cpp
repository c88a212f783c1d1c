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
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <chrono>
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

class Comm {
 public:
  Comm(int nranks, int rank, py::bytes uid, int device, double timeout_s)
      : nranks_(nranks), rank_(rank), device_(device) {
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
        destroy();
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
      destroy();
      throw InitTimeout("ncclCommInitRankConfig: rank " + std::to_string(rank) + " of " + std::to_string(nranks) +
                        " not joined by all peers within " + std::to_string(timeout_s) + " s (aborted)");
    }
    if (state != ncclSuccess) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
      destroy();
      nccl_check(state, "ncclCommInitRankConfig (async)");
    }
  }

  ~Comm() { destroy(); }

  void destroy() {
    if (comm_) {
      hipStreamSynchronize(stream_);
      // non-blocking communicator: finalize (flush) and let it settle before the destroy
      ncclResult_t st = ncclCommFinalize(comm_);
      while (st == ncclInProgress) {
        std::this_thread::yield();
        if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) break;
      }
      ncclCommDestroy(comm_);
      comm_ = nullptr;
    }
    if (stream_) {
      hipEventDestroy(ready_);
      hipEventDestroy(done_);
      hipStreamDestroy(stream_);
      stream_ = nullptr;
    }
  }

  void abort() {
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }

  // comm stream waits for the work already queued on the compute stream
  void after(uint64_t compute) {
    live();
    hip_check(hipEventRecord(ready_, S(compute)), "hipEventRecord");
    hip_check(hipStreamWaitEvent(stream_, ready_, 0), "hipStreamWaitEvent");
  }

  void all_reduce(uint64_t buf, size_t count, int dtype, int op, uint64_t compute) {
    after(compute);
    settle(ncclAllReduce(P(buf), P(buf), count, dtype_of(dtype), op_of(op), comm_, stream_), "ncclAllReduce");
  }

  void broadcast(uint64_t buf, size_t count, int dtype, int root, uint64_t compute) {
    after(compute);
    settle(ncclBroadcast(P(buf), P(buf), count, dtype_of(dtype), root, comm_, stream_), "ncclBroadcast");
  }

  void reduce_scatter(uint64_t send, uint64_t recv, size_t recvcount, int dtype, int op, uint64_t compute) {
    after(compute);
    settle(ncclReduceScatter(P(send), P(recv), recvcount, dtype_of(dtype), op_of(op), comm_, stream_),
           "ncclReduceScatter");
  }

  void all_gather(uint64_t send, uint64_t recv, size_t sendcount, int dtype, uint64_t compute) {
    after(compute);
    settle(ncclAllGather(P(send), P(recv), sendcount, dtype_of(dtype), comm_, stream_), "ncclAllGather");
  }

  // compute stream waits for every collective issued so far
  void join(uint64_t compute) {
    live();
    hip_check(hipEventRecord(done_, stream_), "hipEventRecord");
    hip_check(hipStreamWaitEvent(S(compute), done_, 0), "hipStreamWaitEvent");
  }

  void synchronize() {
    py::gil_scoped_release nogil;
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
  }

  // 0 = healthy; otherwise the ncclResult_t of an asynchronous failure (watchdog)
  int async_error() {
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
  // a non-blocking communicator may answer ncclInProgress: the call is enqueued once its
  // state settles (the watchdog aborts a communicator whose peer failed, which ends this)
  void settle(ncclResult_t r, const char* what) {
    if (r == ncclInProgress) {
      py::gil_scoped_release nogil;
      do {
        std::this_thread::yield();
        if (ncclCommGetAsyncError(comm_, &r) != ncclSuccess) break;
      } while (r == ncclInProgress);
    }
    nccl_check(r, what);
  }
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
