// hipps runtime — a thin native RCCL communicator (rccl.h 2.27).
//
// The reference's transport is MPI_COMM_WORLD through mpi4py (mpi_comms.py:11-13).  hipps' sync
// engines normally go through torch.distributed (backend "nccl" = RCCL); this class is the
// direct route for what torch's process group does not expose:
//   * ncclGather (rccl.h:745) -- the PS gather of the sync PS mode in ONE collective;
//   * all-gather-v as grouped ncclSend/ncclRecv at static per-rank offsets (RCCL has no
//     allgatherv; the reference needs one, mpi_comms.py:160-163);
//   * gather-v (grouped ncclRecv at the root) for variable-size object messages;
//   * ncclCommSplit (rccl.h:290) for sub-communicators;
//   * ncclCommGetAsyncError / ncclCommAbort (rccl.h:271, 362): the engines poll for a dead peer
//     and abort the communicator instead of hanging (failure detection).
// Every call enqueues on the given HIP stream (the engines' comm stream) and returns at once.
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include <ATen/ATen.h>
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <rccl/rccl.h>
#include <torch/extension.h>

namespace py = pybind11;

namespace hipps {
namespace rt {

static void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

static ncclDataType_t dtype_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kDouble: return ncclFloat64;
    default: throw std::runtime_error("unsupported dtype for RCCL");
  }
}

static void dev_contig(const at::Tensor& t, const char* name) {
  if (!t.is_cuda() || !t.is_contiguous()) throw std::runtime_error(std::string(name) + " must be a contiguous device tensor");
}

class RcclComm {
 public:
  static py::bytes unique_id() {
    ncclUniqueId id;
    nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
  }

  RcclComm(py::bytes id_bytes, int nranks, int rank) : nranks_(nranks), rank_(rank) {
    std::string s = id_bytes;
    if ((int)s.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("bad RCCL unique id");
    ncclUniqueId id;
    std::memcpy(id.internal, s.data(), NCCL_UNIQUE_ID_BYTES);
    py::gil_scoped_release nogil;
    nccl_check(ncclCommInitRank(&comm_, nranks, id, rank), "ncclCommInitRank");
  }
  explicit RcclComm(ncclComm_t c) : comm_(c) {
    nccl_check(ncclCommCount(c, &nranks_), "ncclCommCount");
    nccl_check(ncclCommUserRank(c, &rank_), "ncclCommUserRank");
  }
  ~RcclComm() {
    if (comm_) ncclCommDestroy(comm_);
  }

  // collective over this communicator; returns None for ranks that pass color < 0
  std::unique_ptr<RcclComm> split(int color, int key) {
    ncclComm_t nc = nullptr;
    {
      py::gil_scoped_release nogil;
      nccl_check(ncclCommSplit(live(), color < 0 ? NCCL_SPLIT_NOCOLOR : color, key, &nc, nullptr), "ncclCommSplit");
    }
    if (nc == nullptr) return nullptr;
    return std::make_unique<RcclComm>(nc);
  }

  void all_gather(at::Tensor send, at::Tensor recv, uint64_t stream) {
    dev_contig(send, "send");
    dev_contig(recv, "recv");
    if (recv.numel() != send.numel() * nranks_) throw std::runtime_error("all_gather: recv must hold nranks * send");
    nccl_check(ncclAllGather(send.data_ptr(), recv.data_ptr(), send.numel(), dtype_of(send), live(), st(stream)),
               "ncclAllGather");
  }

  // variable-size all-gather: rank r's send lands at recv[displs[r] : displs[r] + counts[r]]
  void all_gather_v(at::Tensor send, at::Tensor recv, const std::vector<int64_t>& counts,
                    const std::vector<int64_t>& displs, uint64_t stream) {
    dev_contig(send, "send");
    dev_contig(recv, "recv");
    if ((int)counts.size() != nranks_ || (int)displs.size() != nranks_) throw std::runtime_error("counts/displs size");
    if (counts[rank_] != send.numel()) throw std::runtime_error("all_gather_v: send size != counts[rank]");
    const size_t es = send.element_size();
    auto dt = dtype_of(send);
    char* rb = static_cast<char*>(recv.data_ptr());
    for (int r = 0; r < nranks_; ++r)
      if (displs[r] + counts[r] > recv.numel()) throw std::runtime_error("all_gather_v: recv too small");
    nccl_check(ncclGroupStart(), "ncclGroupStart");
    for (int r = 0; r < nranks_; ++r) {
      if (r == rank_) continue;
      if (counts[rank_]) nccl_check(ncclSend(send.data_ptr(), counts[rank_], dt, r, live(), st(stream)), "ncclSend");
      if (counts[r]) nccl_check(ncclRecv(rb + displs[r] * es, counts[r], dt, r, live(), st(stream)), "ncclRecv");
    }
    nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    if (counts[rank_])
      hip_ok(hipMemcpyAsync(rb + displs[rank_] * es, send.data_ptr(), counts[rank_] * es, hipMemcpyDeviceToDevice,
                            st(stream)));
  }

  // variable-size gather to root: rank r's send lands at root's recv[displs[r] : + counts[r]]
  // (the reference's Igatherv with exact counts, mpi_comms.py:88, without its padded slots)
  void gather_v(at::Tensor send, c10::optional<at::Tensor> recv, const std::vector<int64_t>& counts,
                const std::vector<int64_t>& displs, int root, uint64_t stream) {
    dev_contig(send, "send");
    if ((int)counts.size() != nranks_ || (int)displs.size() != nranks_) throw std::runtime_error("counts/displs size");
    if (counts[rank_] != send.numel()) throw std::runtime_error("gather_v: send size != counts[rank]");
    const size_t es = send.element_size();
    auto dt = dtype_of(send);
    if (rank_ != root) {
      if (counts[rank_]) nccl_check(ncclSend(send.data_ptr(), counts[rank_], dt, root, live(), st(stream)), "ncclSend");
      return;
    }
    if (!recv.has_value() || !recv->defined()) throw std::runtime_error("gather_v: root needs recv");
    dev_contig(*recv, "recv");
    if (recv->element_size() != (int64_t)es) throw std::runtime_error("gather_v: dtype mismatch");
    char* rb = static_cast<char*>(recv->data_ptr());
    for (int r = 0; r < nranks_; ++r)
      if (displs[r] + counts[r] > recv->numel()) throw std::runtime_error("gather_v: recv too small");
    nccl_check(ncclGroupStart(), "ncclGroupStart");
    for (int r = 0; r < nranks_; ++r)
      if (r != rank_ && counts[r])
        nccl_check(ncclRecv(rb + displs[r] * es, counts[r], dt, r, live(), st(stream)), "ncclRecv");
    nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    if (counts[rank_])
      hip_ok(hipMemcpyAsync(rb + displs[rank_] * es, send.data_ptr(), counts[rank_] * es, hipMemcpyDeviceToDevice,
                            st(stream)));
  }

  void gather(at::Tensor send, c10::optional<at::Tensor> recv, int root, uint64_t stream) {
    dev_contig(send, "send");
    void* rp = nullptr;
    if (rank_ == root) {
      if (!recv.has_value() || !recv->defined()) throw std::runtime_error("gather: root needs recv");
      dev_contig(*recv, "recv");
      if (recv->numel() != send.numel() * nranks_) throw std::runtime_error("gather: recv must hold nranks * send");
      rp = recv->data_ptr();
    }
    nccl_check(ncclGather(send.data_ptr(), rp, send.numel(), dtype_of(send), root, live(), st(stream)), "ncclGather");
  }

  void broadcast(at::Tensor buf, int root, uint64_t stream) {
    dev_contig(buf, "buf");
    nccl_check(ncclBroadcast(buf.data_ptr(), buf.data_ptr(), buf.numel(), dtype_of(buf), root, live(), st(stream)),
               "ncclBroadcast");
  }

  void all_reduce_sum(at::Tensor buf, uint64_t stream) {
    dev_contig(buf, "buf");
    nccl_check(ncclAllReduce(buf.data_ptr(), buf.data_ptr(), buf.numel(), dtype_of(buf), ncclSum, live(), st(stream)),
               "ncclAllReduce");
  }

  void send(at::Tensor buf, int peer, uint64_t stream) {
    dev_contig(buf, "buf");
    nccl_check(ncclSend(buf.data_ptr(), buf.numel(), dtype_of(buf), peer, live(), st(stream)), "ncclSend");
  }

  void recv(at::Tensor buf, int peer, uint64_t stream) {
    dev_contig(buf, "buf");
    nccl_check(ncclRecv(buf.data_ptr(), buf.numel(), dtype_of(buf), peer, live(), st(stream)), "ncclRecv");
  }

  static void group_start() { nccl_check(ncclGroupStart(), "ncclGroupStart"); }
  static void group_end() { nccl_check(ncclGroupEnd(), "ncclGroupEnd"); }

  // 0 = healthy; otherwise the ncclResult_t of the asynchronous failure (peer lost, ...)
  int async_error() {
    if (!comm_) return (int)ncclInvalidUsage;
    ncclResult_t e = ncclSuccess;
    ncclResult_t r = ncclCommGetAsyncError(comm_, &e);
    if (r != ncclSuccess) return (int)r;
    return e == ncclInProgress ? 0 : (int)e;
  }
  std::string error_string(int code) { return ncclGetErrorString((ncclResult_t)code); }

  void abort() {
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }
  void destroy() {
    if (comm_) {
      py::gil_scoped_release nogil;
      ncclCommDestroy(comm_);
      comm_ = nullptr;
    }
  }
  int rank() const { return rank_; }
  int size() const { return nranks_; }
  bool alive() const { return comm_ != nullptr; }
  static int version() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  }

 private:
  ncclComm_t live() {
    if (!comm_) throw std::runtime_error("RCCL communicator was aborted or destroyed");
    return comm_;
  }
  static hipStream_t st(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }
  static void hip_ok(hipError_t e) {
    if (e != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e));
  }
  ncclComm_t comm_ = nullptr;
  int nranks_ = 0, rank_ = 0;
};

void bind_rccl(py::module& m) {
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init<py::bytes, int, int>(), py::arg("unique_id"), py::arg("nranks"), py::arg("rank"))
      .def_static("unique_id", &RcclComm::unique_id)
      .def_static("version", &RcclComm::version)
      .def_static("group_start", &RcclComm::group_start)
      .def_static("group_end", &RcclComm::group_end)
      .def("split", &RcclComm::split, py::arg("color"), py::arg("key"))
      .def("all_gather", &RcclComm::all_gather)
      .def("all_gather_v", &RcclComm::all_gather_v)
      .def("gather", &RcclComm::gather, py::arg("send"), py::arg("recv"), py::arg("root"), py::arg("stream"))
      .def("gather_v", &RcclComm::gather_v, py::arg("send"), py::arg("recv"), py::arg("counts"), py::arg("displs"),
           py::arg("root"), py::arg("stream"))
      .def("broadcast", &RcclComm::broadcast)
      .def("all_reduce_sum", &RcclComm::all_reduce_sum)
      .def("send", &RcclComm::send)
      .def("recv", &RcclComm::recv)
      .def("async_error", &RcclComm::async_error)
      .def("error_string", &RcclComm::error_string)
      .def("abort", &RcclComm::abort)
      .def("destroy", &RcclComm::destroy)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def_property_readonly("alive", &RcclComm::alive);
}

}  // namespace rt
}  // namespace hipps
