// hipps runtime — mailbox memory shared between the PS process and its workers.
//
//   DeviceMailbox : hipMalloc on the PS GPU, exported with hipIpcGetMemHandle (dmabuf IPC on
//                   this stack; HSA_ENABLE_IPC_MODE_LEGACY=0) and mapped by each worker with
//                   hipIpcOpenMemHandle.  Workers then push gradients into it and pull published
//                   parameters out of it with plain stream-ordered D2D copies over xGMI -- a
//                   one-sided transport: nothing on the PS has to post a matching receive, so no
//                   RCCL kernel ever spins on a CU waiting for a straggler.
//   HostMailbox   : the same contract on POSIX shared memory, for CPU-only runs and tests.
//
// Both hand out torch uint8 tensors that alias the mapping (no copies, no deleter: the Python
// object owns the lifetime).
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>
#include <string>

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


void bind_ipc(py::module& m) {
  py::class_<DeviceMailbox>(m, "DeviceMailbox")
      .def(py::init<int64_t>(), py::arg("nbytes"))
      .def(py::init<py::bytes, int64_t>(), py::arg("handle"), py::arg("nbytes"))
      .def("handle", &DeviceMailbox::handle)
      .def("tensor", &DeviceMailbox::tensor)
      .def("close", &DeviceMailbox::close)
      .def_property_readonly("nbytes", &DeviceMailbox::nbytes)
      .def_property_readonly("device", &DeviceMailbox::device);
  py::class_<HostMailbox>(m, "HostMailbox")
      .def(py::init<const std::string&, int64_t, bool>(), py::arg("name"), py::arg("nbytes"), py::arg("create"))
      .def("tensor", &HostMailbox::tensor)
      .def("close", &HostMailbox::close)
      .def("unlink", &HostMailbox::unlink)
      .def_property_readonly("nbytes", &HostMailbox::nbytes);
}

}  // namespace rt
}  // namespace hipps
