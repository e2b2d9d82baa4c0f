// hipps runtime — the async PS control block (see control.cpp for the protocol).  Shared by
// the Python bindings (control.cpp) and the native PS loop (psloop.cpp).
#pragma once
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
#include <tuple>
#include <vector>

#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime/doorbell.h"

namespace py = pybind11;


namespace hipps {
namespace rt {

constexpr int64_t kMagic = 0x5350504948ll;  // "HIPPS"
constexpr int kMaxRanks = 64;
constexpr int kSlots = 64;  // max mailbox slots per worker (bucket messages in flight)
constexpr int kPub = 4;    // published parameter buffers (>= 2 + concurrent readers of old versions)
constexpr int kMaxBuckets = 256;  // bucket-granular publication (ps_granularity='bucket')

struct alignas(64) RankRec {
  std::atomic<int64_t> push_seq;           // last message fully landed in the PS mailbox
  std::atomic<int64_t> ack_seq;            // last message the PS finished reading
  std::atomic<int64_t> push_ver[kSlots];   // param version a slot's gradient was computed on
  std::atomic<int64_t> applied_ver;        // version the worker adopted last
  std::atomic<int64_t> stop;               // worker has finished (seq of its last push)
  std::atomic<int64_t> heartbeat_ns;
  std::atomic<int64_t> incl_seq;           // newest own message reflected in the published params
  std::atomic<int64_t> push_flag[kSlots];  // bucket << 1 | 1 if a presence mask follows (a parameter without a gradient)
  std::atomic<int64_t> reading;            // version whose publish buffer this rank is copying (-1 none)
  std::atomic<int64_t> pull_req;           // p2p transport: parameter requests posted by this worker
  std::atomic<int64_t> sent_ver;           // p2p transport: version the PS sent for the last request
  std::atomic<int64_t> last_stale;         // staleness (updates) of this worker's newest consumed step
  std::atomic<int64_t> last_stale_seq;     // ... and that step's last message seq
  std::atomic<int64_t> reading_b[kMaxBuckets];  // bucket mode: version of bucket b being copied (-1)
};

struct alignas(64) Header {
  int64_t magic;
  int64_t world;
  std::atomic<int64_t> pub_ver;
  std::atomic<int64_t> ps_stop;
  std::atomic<int64_t> error;
  std::atomic<int64_t> drops;
  std::atomic<int64_t> updates;
  std::atomic<int64_t> open_turn;   // staggered mailbox imports: ranks 1..open_turn have mapped
  std::atomic<int64_t> ps_hb;       // PS loop liveness (steady-clock ns), refreshed by its waits
  std::atomic<int64_t> ps_dead_ns;  // workers' waits fail once ps_hb is older than this (0 = never)
  std::atomic<int64_t> buf_ver[kPub + 1];
  std::atomic<int64_t> bpub_ver[kMaxBuckets];        // bucket mode: newest published version of bucket b
  std::atomic<int64_t> bbuf_ver[kMaxBuckets][kPub];  // bucket mode: version in publish slot k of bucket b
  RankRec rank[kMaxRanks];
};

enum Field : int {
  PUSH_SEQ = 0, ACK_SEQ = 1, PUSH_VER = 2, APPLIED_VER = 3, STOP = 4, HEARTBEAT = 5, INCL_SEQ = 6,
  PUSH_FLAG = 7, READING = 8, PULL_REQ = 9, PUB_VER = 10, PS_STOP = 11, ERROR = 12, DROPS = 13, UPDATES = 14, BUF_VER = 15, SENT_VER = 16,
  LAST_STALE = 17, LAST_STALE_SEQ = 18, BPUB_VER = 19, BBUF_VER = 20, READING_B = 21, OPEN_TURN = 22,
  PS_HB = 23, PS_DEAD_NS = 24
};

inline int64_t now_ns() {
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
      for (int r = 0; r < kMaxRanks; ++r) {
        h_->rank[r].reading.store(-1);
        for (int b = 0; b < kMaxBuckets; ++b) h_->rank[r].reading_b[b].store(-1);
      }
      for (int b = 0; b < kMaxBuckets; ++b) {
        h_->bpub_ver[b].store(-1);
        for (int k = 0; k < kPub; ++k) h_->bbuf_ver[b][k].store(-1);
      }
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
    if (dev_) hipHostUnregister(h_);
    if (h_) munmap(h_, sizeof(Header));
  }

  // Register the mapping with HIP so doorbell kernels can store into it.  Returns false (and
  // keeps the host-callback doorbells) if the runtime refuses.
  bool enable_device_doorbells() {
    if (dev_) return true;
    if (hipHostRegister(h_, sizeof(Header), hipHostRegisterMapped | hipHostRegisterPortable) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h_, 0) != hipSuccess || d == nullptr) {
      (void)hipGetLastError();
      hipHostUnregister(h_);
      return false;
    }
    dev_ = reinterpret_cast<char*>(d);
    return true;
  }
  std::string bell_mode() const { return dev_ ? "device" : "host"; }

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
      case PUSH_FLAG: return &rec(idx / kSlots).push_flag[idx % kSlots];
      case READING: return &rec(idx).reading;
      case PULL_REQ: return &rec(idx).pull_req;
      case SENT_VER: return &rec(idx).sent_ver;
      case LAST_STALE: return &rec(idx).last_stale;
      case LAST_STALE_SEQ: return &rec(idx).last_stale_seq;
      case PUB_VER: return &h_->pub_ver;
      case PS_STOP: return &h_->ps_stop;
      case ERROR: return &h_->error;
      case DROPS: return &h_->drops;
      case UPDATES: return &h_->updates;
      case OPEN_TURN: return &h_->open_turn;
      case PS_HB: return &h_->ps_hb;
      case PS_DEAD_NS: return &h_->ps_dead_ns;
      case BUF_VER:
        if (idx < 0 || idx > kPub) throw std::out_of_range("buf_ver index");
        return &h_->buf_ver[idx];
      case BPUB_VER:
        if (idx < 0 || idx >= kMaxBuckets) throw std::out_of_range("bucket index");
        return &h_->bpub_ver[idx];
      case BBUF_VER:  // idx = bucket * kPub + slot
        if (idx < 0 || idx >= kMaxBuckets * kPub) throw std::out_of_range("bucket slot index");
        return &h_->bbuf_ver[idx / kPub][idx % kPub];
      case READING_B:  // idx = rank * kMaxBuckets + bucket
        return &rec(idx / kMaxBuckets).reading_b[idx % kMaxBuckets];
    }
    throw std::out_of_range("unknown control field");
  }

  // seq_cst: the reader/writer handshake on publish buffers (reading vs buf_ver) is Dekker-style
  int64_t load(int field, int idx) { return word(field, idx)->load(std::memory_order_seq_cst); }
  void store(int field, int idx, int64_t v) { word(field, idx)->store(v, std::memory_order_seq_cst); }

  // Block (GIL released) until no rank is reading the publish buffer that holds version v.
  bool wait_no_reader(int64_t v, int64_t timeout_us) {
    py::gil_scoped_release nogil;
    return wait_no_reader_raw(v, timeout_us);
  }
  bool wait_no_reader_raw(int64_t v, int64_t timeout_us) {
    const int64_t deadline = now_ns() + timeout_us * 1000;
    int spins = 0;
    for (;;) {
      ps_beat();
      bool busy = false;
      for (int r = 0; r < (int)h_->world; ++r)
        if (h_->rank[r].reading.load(std::memory_order_seq_cst) == v) busy = true;
      if (!busy) return true;
      if (h_->error.load(std::memory_order_relaxed) || now_ns() >= deadline) return false;
      if (++spins < 2000) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      } else {
        struct timespec ts{0, 20000};
        nanosleep(&ts, nullptr);
      }
    }
  }
  // Bucket mode: block until no rank is reading bucket b at version v.
  bool wait_no_reader_b(int b, int64_t v, int64_t timeout_us) {
    py::gil_scoped_release nogil;
    return wait_no_reader_b_raw(b, v, timeout_us);
  }
  bool wait_no_reader_b_raw(int b, int64_t v, int64_t timeout_us) {
    if (b < 0 || b >= kMaxBuckets) throw std::out_of_range("bucket index");
    const int64_t deadline = now_ns() + timeout_us * 1000;
    int spins = 0;
    for (;;) {
      ps_beat();
      bool busy = false;
      for (int r = 0; r < (int)h_->world; ++r)
        if (h_->rank[r].reading_b[b].load(std::memory_order_seq_cst) == v) busy = true;
      if (!busy) return true;
      if (h_->error.load(std::memory_order_relaxed) || now_ns() >= deadline) return false;
      if (++spins < 2000) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      } else {
        struct timespec ts{0, 20000};
        nanosleep(&ts, nullptr);
      }
    }
  }
  int64_t fetch_add(int field, int idx, int64_t v) { return word(field, idx)->fetch_add(v, std::memory_order_acq_rel); }

  // Block (GIL released) until any rank's push_seq exceeds seen[rank] or PS_STOP / timeout.
  std::vector<int> wait_any(const std::vector<int64_t>& seen, int64_t timeout_us) {
    py::gil_scoped_release nogil;
    return wait_any_raw(seen, timeout_us);
  }
  std::vector<int> wait_any_raw(const std::vector<int64_t>& seen, int64_t timeout_us) {
    const int64_t deadline = now_ns() + timeout_us * 1000;
    const int W = (int)seen.size();
    int spins = 0;
    for (;;) {
      ps_beat();
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
    return wait_ge_raw(field, idx, value, timeout_us);
  }
  bool wait_ge_raw(int field, int idx, int64_t value, int64_t timeout_us) {
    auto* w = word(field, idx);
    const int64_t deadline = now_ns() + timeout_us * 1000;
    int spins = 0;
    while (w->load(std::memory_order_acquire) < value) {
      if (h_->error.load(std::memory_order_relaxed)) return false;
      if (timeout_us >= 0 && now_ns() >= deadline) return false;
      if ((spins & 1023) == 1023 && ps_silent()) return false;
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
    std::atomic<int64_t>* w[kMaxBell];
    int64_t v[kMaxBell];
    int n;
  };
  static void store_cb(void* arg) {
    auto* p = reinterpret_cast<StorePayload*>(arg);
    for (int i = 0; i < p->n; ++i) p->w[i]->store(p->v[i], std::memory_order_release);
    delete p;
  }

  // Stream-ordered doorbell: stores (field, idx, value) triples, in order, after every earlier
  // operation on `stream` has completed.
  // `srcs` (device doorbells only): per word, a device address whose int64 value is stored
  // instead of the immediate (0 = immediate), e.g. the parameter version the GPU adopted.
  void enqueue(uint64_t stream, const std::vector<std::tuple<int, int, int64_t>>& words,
               const std::vector<int64_t>& srcs = {}) {
    if (words.empty()) return;
    if ((int)words.size() > kMaxBell) throw std::runtime_error("too many words for one doorbell");
    auto s = reinterpret_cast<hipStream_t>(stream);
    if (!srcs.empty() && !dev_) throw std::runtime_error("indirect doorbell values need device doorbells");
    if (dev_) {
      DoorbellArgs a{};
      a.n = (int)words.size();
      for (int i = 0; i < a.n; ++i) {
        a.w[i] = dev_word(std::get<0>(words[i]), std::get<1>(words[i]));
        a.v[i] = std::get<2>(words[i]);
        a.src[i] = i < (int)srcs.size() ? reinterpret_cast<const int64_t*>(srcs[i]) : nullptr;
      }
      hipError_t e = launch_doorbell(s, a);
      if (e != hipSuccess) throw std::runtime_error(std::string("doorbell launch failed: ") + hipGetErrorString(e));
      return;
    }
    auto* p = new StorePayload{};
    p->n = (int)words.size();
    for (int i = 0; i < p->n; ++i) {
      p->w[i] = word(std::get<0>(words[i]), std::get<1>(words[i]));
      p->v[i] = std::get<2>(words[i]);
    }
    hipError_t e = hipLaunchHostFunc(s, &ControlBlock::store_cb, p);
    if (e != hipSuccess) {
      delete p;
      throw std::runtime_error(std::string("hipLaunchHostFunc failed: ") + hipGetErrorString(e));
    }
  }

  int64_t* dev_word(int field, int idx) {
    if (!dev_) return nullptr;
    auto* hw = word(field, idx);
    return reinterpret_cast<int64_t*>(dev_ + (reinterpret_cast<char*>(hw) - reinterpret_cast<char*>(h_)));
  }
  int64_t device_addr(int field, int idx) { return reinterpret_cast<int64_t>(dev_word(field, idx)); }

  void enqueue_store(uint64_t stream, int field, int idx, int64_t value) { enqueue(stream, {{field, idx, value}}); }
  void enqueue_store2(uint64_t stream, int f1, int i1, int64_t v1, int f2, int i2, int64_t v2) {
    enqueue(stream, {{f1, i1, v1}, {f2, i2, v2}});
  }

  void heartbeat(int rank) { rec(rank).heartbeat_ns.store(now_ns(), std::memory_order_relaxed); }
  // The PS loop's own liveness word: every PS-side wait refreshes it, and a worker's wait_ge gives
  // up once it is older than ps_dead_ns (the PS thread exited, hung or its process died), so a
  // worker raises within dead_after_s instead of waiting out comm_timeout_s.
  void ps_beat() { h_->ps_hb.store(now_ns(), std::memory_order_relaxed); }
  bool ps_silent() {
    const int64_t lim = h_->ps_dead_ns.load(std::memory_order_relaxed);
    const int64_t hb = h_->ps_hb.load(std::memory_order_relaxed);
    return lim > 0 && hb > 0 && now_ns() - hb > lim;
  }
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
  char* dev_ = nullptr;  // device view of h_ (registered), or null for host-callback doorbells
};

}  // namespace rt
}  // namespace hipps
