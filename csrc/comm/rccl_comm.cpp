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
// Comm(nranks, rank, id, device) -> ncclCommInitRank.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

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

class Comm {
 public:
  Comm(int nranks, int rank, py::bytes uid, int device) : nranks_(nranks), rank_(rank), device_(device) {
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
    {
      py::gil_scoped_release nogil;  // init blocks until every rank joined
      nccl_check(ncclCommInitRank(&comm_, nranks, id, rank), "ncclCommInitRank");
    }
  }

  ~Comm() { destroy(); }

  void destroy() {
    if (comm_) {
      hipStreamSynchronize(stream_);
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
    nccl_check(ncclAllReduce(P(buf), P(buf), count, dtype_of(dtype), op_of(op), comm_, stream_), "ncclAllReduce");
  }

  void broadcast(uint64_t buf, size_t count, int dtype, int root, uint64_t compute) {
    after(compute);
    nccl_check(ncclBroadcast(P(buf), P(buf), count, dtype_of(dtype), root, comm_, stream_), "ncclBroadcast");
  }

  void reduce_scatter(uint64_t send, uint64_t recv, size_t recvcount, int dtype, int op, uint64_t compute) {
    after(compute);
    nccl_check(ncclReduceScatter(P(send), P(recv), recvcount, dtype_of(dtype), op_of(op), comm_, stream_),
               "ncclReduceScatter");
  }

  void all_gather(uint64_t send, uint64_t recv, size_t sendcount, int dtype, uint64_t compute) {
    after(compute);
    nccl_check(ncclAllGather(P(send), P(recv), sendcount, dtype_of(dtype), comm_, stream_), "ncclAllGather");
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
  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  int device() const { return device_; }

 private:
  void live() const {
    if (!comm_) throw std::runtime_error("communicator destroyed or aborted");
  }
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
  py::class_<Comm>(m, "Comm")
      .def(py::init<int, int, py::bytes, int>(), py::arg("nranks"), py::arg("rank"), py::arg("uid"),
           py::arg("device"))
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
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("nranks", &Comm::nranks)
      .def_property_readonly("device", &Comm::device);
}
