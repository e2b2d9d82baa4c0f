// hipps runtime — mailbox memory shared between the PS process and its workers.
//
//   DeviceMailbox : hipMalloc on the PS GPU, exported with hipIpcGetMemHandle (dmabuf IPC on
//                   this stack; HSA_ENABLE_IPC_MODE_LEGACY=0) and mapped by each worker with
//                   hipIpcOpenMemHandle.  Workers then push gradients into it and pull published
//                   parameters out of it with plain stream-ordered D2D copies over xGMI -- a
//                   one-sided transport: nothing on the PS has to post a matching receive, so no
//                   RCCL kernel ever spins on a CU waiting for a straggler.
//   VmmRegion     : the same mailbox built from the virtual-memory API instead (hipMemCreate
//                   chunks mapped back to back into one reserved VA range): each chunk is exported
//                   as a POSIX fd (dmabuf), the fds travel to the worker over a Unix socket
//                   (SCM_RIGHTS), and the worker maps them back to back into its own VA range --
//                   the region stays contiguous on both sides while no single import is larger
//                   than one chunk (a multi-GB hipIpcOpenMemHandle sometimes never returned on the
//                   rehearsal box: profiles/r5/ipc).
//   HostMailbox   : the same contract on POSIX shared memory, for CPU-only runs and tests.
//
// Both hand out torch uint8 tensors that alias the mapping (no copies, no deleter: the Python
// object owns the lifetime).
#include <fcntl.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include <ATen/ATen.h>
#include <c10/hip/HIPFunctions.h>
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <torch/extension.h>

namespace py = pybind11;

namespace hipps {
namespace rt {

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

class DeviceMailbox {
 public:
  // create: allocate `nbytes` on the current device
  DeviceMailbox(int64_t nbytes) : nbytes_(nbytes), owner_(true) {
    hip_check(hipGetDevice(&device_), "hipGetDevice");
    hip_check(hipMalloc(&ptr_, (size_t)nbytes), "hipMalloc(mailbox)");
    hip_check(hipMemset(ptr_, 0, (size_t)nbytes), "hipMemset(mailbox)");
  }
  // open: map a peer's exported allocation on the current device
  DeviceMailbox(py::bytes handle, int64_t nbytes) : nbytes_(nbytes), owner_(false) {
    std::string h = handle;
    if (h.size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("bad IPC handle size");
    hipIpcMemHandle_t mh;
    std::memcpy(&mh, h.data(), sizeof(mh));
    hip_check(hipGetDevice(&device_), "hipGetDevice");
    hipError_t e;
    {
      // without the GIL: a Python-side guard can still run if the driver call never returns
      py::gil_scoped_release nogil;
      e = hipIpcOpenMemHandle(&ptr_, mh, hipIpcMemLazyEnablePeerAccess);
    }
    hip_check(e, "hipIpcOpenMemHandle");
  }
  ~DeviceMailbox() { close(); }

  void close() {
    if (!ptr_) return;
    hipDeviceSynchronize();
    if (owner_) hipFree(ptr_);
    else hipIpcCloseMemHandle(ptr_);
    ptr_ = nullptr;
  }

  py::bytes handle() const {
    if (!owner_) throw std::runtime_error("only the allocating process exports the handle");
    hipIpcMemHandle_t mh;
    hip_check(hipIpcGetMemHandle(&mh, ptr_), "hipIpcGetMemHandle");
    return py::bytes(reinterpret_cast<const char*>(&mh), sizeof(mh));
  }

  at::Tensor tensor() const {
    if (!ptr_) throw std::runtime_error("mailbox closed");
    auto opts = at::TensorOptions().dtype(at::kByte).device(at::Device(at::kCUDA, device_));
    return at::from_blob(ptr_, {nbytes_}, opts);
  }

  int64_t nbytes() const { return nbytes_; }
  int device() const { return device_; }

 private:
  void* ptr_ = nullptr;
  int64_t nbytes_;
  int device_ = 0;
  bool owner_;
};

class HostMailbox {
 public:
  HostMailbox(const std::string& name, int64_t nbytes, bool create) : name_(name), nbytes_(nbytes) {
    int fd = shm_open(name.c_str(), create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(" + name + ") failed: " + std::strerror(errno));
    if (create && ftruncate(fd, nbytes) != 0) {
      ::close(fd);
      throw std::runtime_error("ftruncate(mailbox) failed");
    }
    ptr_ = mmap(nullptr, (size_t)nbytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (ptr_ == MAP_FAILED) {
      ptr_ = nullptr;
      throw std::runtime_error("mmap(mailbox) failed");
    }
  }
  ~HostMailbox() { close(); }
  void close() {
    if (ptr_) munmap(ptr_, (size_t)nbytes_);
    ptr_ = nullptr;
  }
  void unlink() { shm_unlink(name_.c_str()); }
  at::Tensor tensor() const {
    if (!ptr_) throw std::runtime_error("mailbox closed");
    return at::from_blob(ptr_, {nbytes_}, at::TensorOptions().dtype(at::kByte));
  }
  int64_t nbytes() const { return nbytes_; }

 private:
  std::string name_;
  int64_t nbytes_;
  void* ptr_ = nullptr;
};


// ---------------------------------------------------------------------------------------------
// VMM region: chunked physical allocations in one contiguous VA range, exportable as POSIX fds
class VmmRegion {
 public:
  // create: nbytes on the current device, in chunks of (about) chunk bytes
  VmmRegion(int64_t nbytes, int64_t chunk) : owner_(true) {
    hip_check(hipGetDevice(&device_), "hipGetDevice");
    hipMemAllocationProp prop = make_prop(device_);
    size_t gran = 0;
    hip_check(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended),
              "hipMemGetAllocationGranularity");
    if (gran == 0) gran = 2 << 20;
    const int64_t g = (int64_t)gran;
    const int64_t ch = ((chunk > 0 ? chunk : nbytes) + g - 1) / g * g;
    total_ = (nbytes + g - 1) / g * g;
    for (int64_t off = 0; off < total_; off += ch) sizes_.push_back(off + ch <= total_ ? ch : total_ - off);
    hip_check(hipMemAddressReserve(&ptr_, (size_t)total_, 0, nullptr, 0), "hipMemAddressReserve");
    int64_t off = 0;
    for (int64_t sz : sizes_) {
      hipMemGenericAllocationHandle_t h;
      hip_check(hipMemCreate(&h, (size_t)sz, &prop, 0), "hipMemCreate");
      handles_.push_back(h);
      hip_check(hipMemMap(reinterpret_cast<char*>(ptr_) + off, (size_t)sz, 0, h, 0), "hipMemMap");
      off += sz;
    }
    set_access();
    hip_check(hipMemset(ptr_, 0, (size_t)total_), "hipMemset(vmm)");
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    nbytes_ = nbytes;
  }
  // import: chunk fds (received over a socket; closed here) mapped back to back on this device
  VmmRegion(std::vector<int> fds, std::vector<int64_t> sizes, int64_t nbytes) : owner_(false) {
    if (fds.size() != sizes.size() || fds.empty()) throw std::runtime_error("VmmRegion: fds / sizes mismatch");
    hip_check(hipGetDevice(&device_), "hipGetDevice");
    sizes_ = sizes;
    total_ = 0;
    for (int64_t s : sizes) total_ += s;
    {
      py::gil_scoped_release nogil;
      hipError_t e = hipMemAddressReserve(&ptr_, (size_t)total_, 0, nullptr, 0);
      int64_t off = 0;
      for (size_t i = 0; i < fds.size() && e == hipSuccess; ++i) {
        hipMemGenericAllocationHandle_t h;
        // HIP reads the fd through the pointer (the CUDA form, the fd value cast to a pointer,
        // dereferenced it as an address: SIGSEGV, profiles/r5/ipc)
        int fd = fds[i];
        e = hipMemImportFromShareableHandle(&h, &fd, hipMemHandleTypePosixFileDescriptor);
        if (e != hipSuccess) break;
        handles_.push_back(h);
        e = hipMemMap(reinterpret_cast<char*>(ptr_) + off, (size_t)sizes[i], 0, h, 0);
        off += sizes[i];
      }
      // the fds stay open until release(): a chunk's fd number is not handed out again while
      // its import is mapped (a re-import in the same process once saw another allocation's
      // pages when the numbers were recycled, profiles/r5/ipc)
      fds_ = fds;
      if (e != hipSuccess) {
        release();
        hip_check(e, "VmmRegion import");
      }
    }
    set_access();
    nbytes_ = nbytes;
  }
  ~VmmRegion() { close(); }

  // fresh fds of every chunk (the caller sends and closes them)
  std::vector<int> export_fds() const {
    if (!owner_) throw std::runtime_error("only the allocating process exports");
    std::vector<int> out;
    for (auto h : handles_) {
      int fd = -1;
      hip_check(hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0),
                "hipMemExportToShareableHandle");
      out.push_back(fd);
    }
    return out;
  }
  std::vector<int64_t> chunk_sizes() const { return sizes_; }

  at::Tensor tensor() const {
    if (!ptr_) throw std::runtime_error("region closed");
    auto opts = at::TensorOptions().dtype(at::kByte).device(at::Device(at::kCUDA, device_));
    return at::from_blob(ptr_, {nbytes_}, opts);
  }
  void close() {
    if (!ptr_) return;
    hipDeviceSynchronize();
    release();
  }
  int64_t nbytes() const { return nbytes_; }
  int64_t mapped() const { return total_; }
  int nchunks() const { return (int)sizes_.size(); }

 private:
  static hipMemAllocationProp make_prop(int dev) {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.requestedHandleTypes = hipMemHandleTypePosixFileDescriptor;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    return prop;
  }
  void set_access() {
    hipMemAccessDesc d{};
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = device_;
    d.flags = hipMemAccessFlagsProtReadWrite;
    hip_check(hipMemSetAccess(ptr_, (size_t)total_, &d, 1), "hipMemSetAccess");
  }
  void release() {
    if (ptr_) {
      int64_t off = 0;
      for (size_t i = 0; i < handles_.size(); ++i) {
        hipMemUnmap(reinterpret_cast<char*>(ptr_) + off, (size_t)sizes_[i]);
        off += sizes_[i];
      }
      for (auto h : handles_) hipMemRelease(h);
      hipMemAddressFree(ptr_, (size_t)total_);
    }
    handles_.clear();
    for (int fd : fds_) ::close(fd);
    fds_.clear();
    ptr_ = nullptr;
  }
  void* ptr_ = nullptr;
  int64_t nbytes_ = 0, total_ = 0;
  int device_ = 0;
  bool owner_;
  std::vector<int64_t> sizes_;
  std::vector<hipMemGenericAllocationHandle_t> handles_;
  std::vector<int> fds_;  // imported chunks' fds, closed with the mapping
};

// ---------------------------------------------------------------------------------------------
// fd passing over an abstract-namespace Unix socket (SCM_RIGHTS)
static sockaddr_un abstract_addr(const std::string& name, socklen_t* len) {
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  if (name.size() + 1 > sizeof(a.sun_path)) throw std::runtime_error("socket name too long");
  a.sun_path[0] = '\0';
  std::memcpy(a.sun_path + 1, name.data(), name.size());
  *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + name.size());
  return a;
}

class FdServer {
 public:
  explicit FdServer(const std::string& name) {
    fd_ = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd_ < 0) throw std::runtime_error(std::string("socket: ") + std::strerror(errno));
    socklen_t len;
    sockaddr_un a = abstract_addr(name, &len);
    if (::bind(fd_, reinterpret_cast<sockaddr*>(&a), len) != 0 || ::listen(fd_, 64) != 0) {
      const int err = errno;
      ::close(fd_);
      fd_ = -1;
      throw std::runtime_error(std::string("bind/listen ") + name + ": " + std::strerror(err));
    }
  }
  ~FdServer() { close(); }
  void close() {
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
  }
  // accept one client and send it `fds` (then close them); false on timeout
  bool send_one(std::vector<int> fds, int64_t timeout_ms) {
    py::gil_scoped_release nogil;
    pollfd p{fd_, POLLIN, 0};
    const int r = ::poll(&p, 1, (int)timeout_ms);
    if (r <= 0) {
      for (int f : fds) ::close(f);
      return false;
    }
    const int c = ::accept4(fd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (c < 0) {
      for (int f : fds) ::close(f);
      throw std::runtime_error(std::string("accept: ") + std::strerror(errno));
    }
    const int n = (int)fds.size();
    std::vector<char> ctl(CMSG_SPACE(sizeof(int) * n));
    int32_t count = n;
    iovec io{&count, sizeof(count)};
    msghdr m{};
    m.msg_iov = &io;
    m.msg_iovlen = 1;
    m.msg_control = ctl.data();
    m.msg_controllen = ctl.size();
    cmsghdr* cm = CMSG_FIRSTHDR(&m);
    cm->cmsg_level = SOL_SOCKET;
    cm->cmsg_type = SCM_RIGHTS;
    cm->cmsg_len = CMSG_LEN(sizeof(int) * n);
    std::memcpy(CMSG_DATA(cm), fds.data(), sizeof(int) * n);
    const ssize_t w = ::sendmsg(c, &m, 0);
    const int err = errno;
    ::close(c);
    for (int f : fds) ::close(f);
    if (w != (ssize_t)sizeof(count)) throw std::runtime_error(std::string("sendmsg: ") + std::strerror(err));
    return true;
  }

 private:
  int fd_ = -1;
};

static std::vector<int> fd_recv(const std::string& name, int64_t timeout_ms) {
  py::gil_scoped_release nogil;
  socklen_t len;
  sockaddr_un a = abstract_addr(name, &len);
  const auto t0 = std::chrono::steady_clock::now();
  int s = -1;
  for (;;) {  // the server may not listen yet
    s = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (s < 0) throw std::runtime_error(std::string("socket: ") + std::strerror(errno));
    if (::connect(s, reinterpret_cast<sockaddr*>(&a), len) == 0) break;
    ::close(s);
    s = -1;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms))
      throw std::runtime_error("fd_recv: cannot connect to " + name);
    ::usleep(2000);
  }
  std::vector<char> ctl(CMSG_SPACE(sizeof(int) * 250));
  int32_t count = 0;
  iovec io{&count, sizeof(count)};
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = ctl.data();
  m.msg_controllen = ctl.size();
  pollfd p{s, POLLIN, 0};
  if (::poll(&p, 1, (int)timeout_ms) <= 0) {
    ::close(s);
    throw std::runtime_error("fd_recv: no fds from " + name);
  }
  const ssize_t r = ::recvmsg(s, &m, MSG_CMSG_CLOEXEC);
  ::close(s);
  if (r != (ssize_t)sizeof(count)) throw std::runtime_error("fd_recv: short message");
  std::vector<int> out;
  for (cmsghdr* cm = CMSG_FIRSTHDR(&m); cm; cm = CMSG_NXTHDR(&m, cm)) {
    if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_RIGHTS) {
      const int n = (int)((cm->cmsg_len - CMSG_LEN(0)) / sizeof(int));
      const int* f = reinterpret_cast<const int*>(CMSG_DATA(cm));
      out.insert(out.end(), f, f + n);
    }
  }
  if ((int)out.size() != count) throw std::runtime_error("fd_recv: fd count mismatch");
  return out;
}

void bind_ipc(py::module& m) {
  py::class_<DeviceMailbox>(m, "DeviceMailbox")
      .def(py::init<int64_t>(), py::arg("nbytes"))
      .def(py::init<py::bytes, int64_t>(), py::arg("handle"), py::arg("nbytes"))
      .def("handle", &DeviceMailbox::handle)
      .def("tensor", &DeviceMailbox::tensor)
      .def("close", &DeviceMailbox::close)
      .def_property_readonly("nbytes", &DeviceMailbox::nbytes)
      .def_property_readonly("device", &DeviceMailbox::device);
  py::class_<VmmRegion>(m, "VmmRegion")
      .def(py::init<int64_t, int64_t>(), py::arg("nbytes"), py::arg("chunk"))
      .def(py::init<std::vector<int>, std::vector<int64_t>, int64_t>(), py::arg("fds"), py::arg("sizes"),
           py::arg("nbytes"))
      .def("export_fds", &VmmRegion::export_fds)
      .def("chunk_sizes", &VmmRegion::chunk_sizes)
      .def("tensor", &VmmRegion::tensor)
      .def("close", &VmmRegion::close)
      .def_property_readonly("nbytes", &VmmRegion::nbytes)
      .def_property_readonly("mapped", &VmmRegion::mapped)
      .def_property_readonly("nchunks", &VmmRegion::nchunks);
  py::class_<FdServer>(m, "FdServer")
      .def(py::init<const std::string&>(), py::arg("name"))
      .def("send_one", &FdServer::send_one, py::arg("fds"), py::arg("timeout_ms"))
      .def("close", &FdServer::close);
  m.def("fd_recv", &fd_recv, py::arg("name"), py::arg("timeout_ms"));
  py::class_<HostMailbox>(m, "HostMailbox")
      .def(py::init<const std::string&, int64_t, bool>(), py::arg("name"), py::arg("nbytes"), py::arg("create"))
      .def("tensor", &HostMailbox::tensor)
      .def("close", &HostMailbox::close)
      .def("unlink", &HostMailbox::unlink)
      .def_property_readonly("nbytes", &HostMailbox::nbytes);
}

}  // namespace rt
}  // namespace hipps
