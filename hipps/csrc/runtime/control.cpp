// hipps runtime — shared-memory control plane for the asynchronous parameter server.
//
// MPI gives the reference an any-source receive (README.md:65-70 `recv(MPI.ANY_SOURCE)`); RCCL
// has none.  On one node hipps replaces it with a POSIX shared-memory control block: each rank
// owns a cache-line-padded record of sequence words (gradient pushed / consumed, version used,
// stop), and the PS owns the published-parameter version words.  Data never goes through here
// (it moves device-to-device into IPC mailboxes, see ipc.cpp); only 8-byte doorbells do.
//
//   worker: copy grad -> PS mailbox slot (comm stream) ; then hipLaunchHostFunc -> push_seq = s
//   PS:     wait_any(push_seq > seen) ; accumulate slot ; hostfunc -> ack_seq = s
//   PS:     after M grads: update + publish into pub buffer b ; hostfunc -> buf_ver[b], pub_ver
//   worker: irequest_params(): pub_ver newer? copy pub[pub_ver % NPUB] (one-sided pull)
//
// Doorbells written from a stream callback are ordered after the stream's earlier work, so a
// doorbell never runs ahead of the bytes it announces.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

namespace py = pybind11;

namespace hipps {
namespace rt {

constexpr int64_t kMagic = 0x5350504948ll;  // "HIPPS"
constexpr int kMaxRanks = 64;
constexpr int kSlots = 64;  // max mailbox slots per worker (bucket messages in flight)
constexpr int kPub = 3;    // published parameter buffers

struct alignas(64) RankRec {
  std::atomic<int64_t> push_seq;           // last message fully landed in the PS mailbox
  std::atomic<int64_t> ack_seq;            // last message the PS finished reading
  std::atomic<int64_t> push_ver[kSlots];   // param version a slot's gradient was computed on
  std::atomic<int64_t> applied_ver;        // version the worker adopted last
  std::atomic<int64_t> stop;               // worker has finished (seq of its last push)
  std::atomic<int64_t> heartbeat_ns;
  std::atomic<int64_t> incl_seq;           // newest own message reflected in the published params
};

struct alignas(64) Header {
  int64_t magic;
  int64_t world;
  std::atomic<int64_t> pub_ver;
  std::atomic<int64_t> ps_stop;
  std::atomic<int64_t> error;
  std::atomic<int64_t> drops;
  std::atomic<int64_t> updates;
  std::atomic<int64_t> buf_ver[kPub + 1];
  RankRec rank[kMaxRanks];
};

enum Field : int {
  PUSH_SEQ = 0, ACK_SEQ = 1, PUSH_VER = 2, APPLIED_VER = 3, STOP = 4, HEARTBEAT = 5, INCL_SEQ = 6,
  PUB_VER = 10, PS_STOP = 11, ERROR = 12, DROPS = 13, UPDATES = 14, BUF_VER = 15
};

static int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

class ControlBlock {
 public:
  ControlBlock(const std::string& name, int world, bool create) : name_(name), create_(create) {
    if (world < 1 || world > kMaxRanks) throw std::runtime_error("world size out of range for control block");
    int flags = create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR;
    int fd = shm_open(name.c_str(), flags, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(" + name + ") failed: " + std::strerror(errno));
    if (create && ftruncate(fd, sizeof(Header)) != 0) {
      close(fd);
      throw std::runtime_error("ftruncate failed");
    }
    void* p = mmap(nullptr, sizeof(Header), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("mmap of control block failed");
    h_ = reinterpret_cast<Header*>(p);
    if (create) {
      std::memset(p, 0, sizeof(Header));
      h_->world = world;
      for (int b = 0; b <= kPub; ++b) h_->buf_ver[b].store(-1);
      h_->pub_ver.store(-1);
      std::atomic_thread_fence(std::memory_order_release);
      h_->magic = kMagic;
    } else {
      for (int i = 0; i < 2000 && reinterpret_cast<volatile int64_t&>(h_->magic) != kMagic; ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      if (h_->magic != kMagic) throw std::runtime_error("control block " + name + " not initialised");
      if (h_->world != world) throw std::runtime_error("control block world size mismatch");
    }
  }
  ~ControlBlock() {
    if (h_) munmap(h_, sizeof(Header));
  }

  void unlink() { shm_unlink(name_.c_str()); }

  std::atomic<int64_t>* word(int field, int idx) {
    switch (field) {
      case PUSH_SEQ: return &rec(idx).push_seq;
      case ACK_SEQ: return &rec(idx).ack_seq;
      case PUSH_VER: return &rec(idx / kSlots).push_ver[idx % kSlots];
      case APPLIED_VER: return &rec(idx).applied_ver;
      case STOP: return &rec(idx).stop;
      case HEARTBEAT: return &rec(idx).heartbeat_ns;
      case INCL_SEQ: return &rec(idx).incl_seq;
      case PUB_VER: return &h_->pub_ver;
      case PS_STOP: return &h_->ps_stop;
      case ERROR: return &h_->error;
      case DROPS: return &h_->drops;
      case UPDATES: return &h_->updates;
      case BUF_VER:
        if (idx < 0 || idx > kPub) throw std::out_of_range("buf_ver index");
        return &h_->buf_ver[idx];
    }
    throw std::out_of_range("unknown control field");
  }

  int64_t load(int field, int idx) { return word(field, idx)->load(std::memory_order_acquire); }
  void store(int field, int idx, int64_t v) { word(field, idx)->store(v, std::memory_order_release); }
  int64_t fetch_add(int field, int idx, int64_t v) { return word(field, idx)->fetch_add(v, std::memory_order_acq_rel); }

  // Block (GIL released) until any rank's push_seq exceeds seen[rank] or PS_STOP / timeout.
  std::vector<int> wait_any(const std::vector<int64_t>& seen, int64_t timeout_us) {
    py::gil_scoped_release nogil;
    const int64_t deadline = now_ns() + timeout_us * 1000;
    const int W = (int)seen.size();
    int spins = 0;
    for (;;) {
      std::vector<int> ready;
      for (int r = 0; r < W; ++r)
        if (rec(r).push_seq.load(std::memory_order_acquire) > seen[r]) ready.push_back(r);
      if (!ready.empty() || h_->ps_stop.load(std::memory_order_acquire)) return ready;
      if (now_ns() >= deadline) return ready;
      if (++spins < 2000) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      } else {
        struct timespec ts{0, 20000};  // 20 us
        nanosleep(&ts, nullptr);
      }
    }
  }

  // Block (GIL released) until word >= value; returns false on timeout.
  bool wait_ge(int field, int idx, int64_t value, int64_t timeout_us) {
    py::gil_scoped_release nogil;
    auto* w = word(field, idx);
    const int64_t deadline = now_ns() + timeout_us * 1000;
    int spins = 0;
    while (w->load(std::memory_order_acquire) < value) {
      if (h_->error.load(std::memory_order_relaxed)) return false;
      if (timeout_us >= 0 && now_ns() >= deadline) return false;
      if (++spins < 2000) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      } else {
        struct timespec ts{0, 20000};
        nanosleep(&ts, nullptr);
      }
    }
    return true;
  }

  struct StorePayload {
    std::atomic<int64_t>* w;
    int64_t v;
    std::atomic<int64_t>* w2;  // optional second word, stored after the first
    int64_t v2;
  };
  static void store_cb(void* arg) {
    auto* p = reinterpret_cast<StorePayload*>(arg);
    p->w->store(p->v, std::memory_order_release);
    if (p->w2) p->w2->store(p->v2, std::memory_order_release);
    delete p;
  }

  // Stream-ordered doorbell: runs after every earlier operation on `stream` has completed.
  void enqueue_store(uint64_t stream, int field, int idx, int64_t value) {
    auto* p = new StorePayload{word(field, idx), value, nullptr, 0};
    hipError_t e = hipLaunchHostFunc(reinterpret_cast<hipStream_t>(stream), &ControlBlock::store_cb, p);
    if (e != hipSuccess) {
      delete p;
      throw std::runtime_error(std::string("hipLaunchHostFunc failed: ") + hipGetErrorString(e));
    }
  }

  // Two ordered doorbells in one callback (e.g. slot version, then the sequence word).
  void enqueue_store2(uint64_t stream, int f1, int i1, int64_t v1, int f2, int i2, int64_t v2) {
    auto* p = new StorePayload{word(f1, i1), v1, word(f2, i2), v2};
    hipError_t e = hipLaunchHostFunc(reinterpret_cast<hipStream_t>(stream), &ControlBlock::store_cb, p);
    if (e != hipSuccess) {
      delete p;
      throw std::runtime_error(std::string("hipLaunchHostFunc failed: ") + hipGetErrorString(e));
    }
  }

  void heartbeat(int rank) { rec(rank).heartbeat_ns.store(now_ns(), std::memory_order_relaxed); }
  int world() const { return (int)h_->world; }
  static int slots() { return kSlots; }
  static int npub() { return kPub; }

 private:
  RankRec& rec(int r) {
    if (r < 0 || r >= h_->world) throw std::out_of_range("rank out of range");
    return h_->rank[r];
  }
  std::string name_;
  bool create_;
  Header* h_ = nullptr;
};

void bind_control(py::module& m) {
  py::class_<ControlBlock>(m, "ControlBlock")
      .def(py::init<const std::string&, int, bool>(), py::arg("name"), py::arg("world"), py::arg("create"))
      .def("unlink", &ControlBlock::unlink)
      .def("load", &ControlBlock::load)
      .def("store", &ControlBlock::store)
      .def("fetch_add", &ControlBlock::fetch_add)
      .def("wait_any", &ControlBlock::wait_any)
      .def("wait_ge", &ControlBlock::wait_ge)
      .def("enqueue_store", &ControlBlock::enqueue_store)
      .def("enqueue_store2", &ControlBlock::enqueue_store2)
      .def("heartbeat", &ControlBlock::heartbeat)
      .def_property_readonly("world", &ControlBlock::world)
      .def_property_readonly_static("SLOTS", [](py::object) { return kSlots; })
      .def_property_readonly_static("NPUB", [](py::object) { return kPub; });
  m.attr("F_PUSH_SEQ") = (int)PUSH_SEQ;
  m.attr("F_ACK_SEQ") = (int)ACK_SEQ;
  m.attr("F_PUSH_VER") = (int)PUSH_VER;
  m.attr("F_APPLIED_VER") = (int)APPLIED_VER;
  m.attr("F_STOP") = (int)STOP;
  m.attr("F_HEARTBEAT") = (int)HEARTBEAT;
  m.attr("F_INCL_SEQ") = (int)INCL_SEQ;
  m.attr("F_PUB_VER") = (int)PUB_VER;
  m.attr("F_PS_STOP") = (int)PS_STOP;
  m.attr("F_ERROR") = (int)ERROR;
  m.attr("F_DROPS") = (int)DROPS;
  m.attr("F_UPDATES") = (int)UPDATES;
  m.attr("F_BUF_VER") = (int)BUF_VER;
}

}  // namespace rt
}  // namespace hipps
