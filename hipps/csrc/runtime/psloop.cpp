// hipps runtime — the AsySG-InCon parameter-server loop as a native thread (no GIL).
//
// The PS of README.md:64-76 (rank 0 receives from ANY_SOURCE, sums M gradients, steps, publishes)
// runs on rank 0 beside worker 0.  Its Python form (ps_async.py _serve + ps_core.PSCore) holds
// the GIL for every message it bookkeeps and every kernel it launches, and that GIL is the one
// worker 0's trainer needs: under an emulated W=8 message load worker 0 lost 8 % (VERDICT r4
// weak #8).  This loop is the same protocol -- per-bucket versions (ps_granularity='bucket'),
// staleness rule, M-accumulation, ordered acks / publish doorbells -- in C++: it waits on the
// control block (control.h), launches the codec's accumulate kernels and the fused optimizer
// kernels on the PS stream through the same C++ entry points the Python path calls, and rings
// the same doorbells.  Python configures it once, pushes the optimizer hyper-parameters at each
// step() and reads its counters back; the Python loop remains for the configurations this one
// does not take (whole-model versions, p2p transport, object codecs, fault injection, probes).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <ATen/ATen.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "runtime/control.h"

namespace hipps {
void aggregate(const std::vector<at::Tensor>& slots, at::Tensor acc, double gscale, bool accumulate, bool acquire);
void copy_acquire(at::Tensor src, at::Tensor dst);
void sgd_step(const std::vector<at::Tensor>& grads, double gscale, at::Tensor p, c10::optional<at::Tensor> buf,
              c10::optional<at::Tensor> pub, bool zero_src, double lr, double wd, double momentum, double dampening,
              bool nesterov, bool first, c10::optional<at::Tensor> mask, c10::optional<at::Tensor> csteps,
              double lookahead);
void adam_step(const std::vector<at::Tensor>& grads, double gscale, at::Tensor p, at::Tensor exp_avg,
               at::Tensor exp_avg_sq, c10::optional<at::Tensor> max_exp_avg_sq, c10::optional<at::Tensor> pub,
               bool zero_src, double lr, double beta1, double beta2, double eps, double wd, int64_t step,
               bool amsgrad, bool torch_mode, c10::optional<at::Tensor> mask, c10::optional<at::Tensor> csteps);
void q8_aggregate(const std::vector<at::Tensor>& qs, const std::vector<at::Tensor>& ss, at::Tensor acc, double gscale,
                  bool accumulate, bool acquire);
void topk_accumulate(at::Tensor idx, at::Tensor val, at::Tensor acc, double gscale, bool acquire);
void topk_q8_accumulate(at::Tensor idx, at::Tensor q, at::Tensor scales, at::Tensor acc, double gscale,
                        bool acquire);
void thresh_accumulate(at::Tensor count, at::Tensor idx, at::Tensor val, at::Tensor acc, double gscale,
                       bool acquire);

namespace rt {
void emu_sweep(at::Tensor wr, at::Tensor rd, at::Tensor sink, int64_t stamp, int64_t blocks);

// codec of a bucket's message (hipps/codecs): which fields, in which order
enum Kind : int { kDense = 0, kQ8 = 1, kTopk = 2, kTopkQ8 = 3, kThresh = 4 };

struct MsgField {
  int64_t off, numel;
  at::ScalarType dtype;
};
struct BucketDesc {
  int64_t lo, hi, msg_ext, wire_off, msg_nbytes;
  int kind;
  std::vector<MsgField> f;
};
struct Group {
  int64_t a, b;
  bool adam;
  double lr, wd, mom, damp, beta1, beta2, eps;
  bool nesterov, amsgrad, torch_mode;
  int64_t steps;  // the optimizer's per-group step counter (_group_steps)
};
struct Pend {
  int bi;
  double scale;
  int worker;
  int64_t off;  // message offset in the worker's ring
  bool emu;     // an emulated remote copy of the preceding message (cfg.emulate_remote)
};

static at::ScalarType dtype_of(int code) {
  switch (code) {
    case 0: return at::kFloat;
    case 1: return at::kBFloat16;
    case 2: return at::kChar;
    case 3: return at::kInt;
    case 4: return at::kByte;
  }
  throw std::runtime_error("native PS: unknown dtype code");
}

class NativePS {
 public:
  NativePS(ControlBlock& ctl, py::dict c) : ctl_(ctl) {
    W_ = c["W"].cast<int>();
    rank_ = c["rank"].cast<int>();
    nb_ = c["nb"].cast<int>();
    SLOTS_ = c["slots"].cast<int>();
    MAXSLOTS_ = c["maxslots"].cast<int>();
    M_ = c["M"].cast<int>();
    staleness_ = c["staleness"].cast<int64_t>();
    staleness_lr_ = c["staleness_lr"].cast<bool>();
    gscale_ = c["gscale"].cast<double>();
    npub_ = c["npub"].cast<int>();
    dead_after_us_ = c["dead_after_us"].cast<int64_t>();
    skip_missing_ = c["skip_missing"].cast<bool>();
    ns_ = c["nslots"].cast<int64_t>();
    device_ = c["device"].cast<int>();
    stream_ = c["stream"].cast<int64_t>();
    direct_ok_ = c["direct_ok"].cast<bool>();
    acc_ = c["acc"].cast<at::Tensor>();
    // per-bucket versions at M = 1: acc_ is one bucket-sized scratch (ps_async._acc_scratch)
    acc_scratch_ = c.contains("acc_scratch") && c["acc_scratch"].cast<bool>();
    master_ = c["master"].cast<at::Tensor>();
    // publish buffers as chunks of pub_chunk elements (each an IPC allocation below 2 GiB), typed
    for (auto q : c["pub_chunks"].cast<py::list>()) {
      std::vector<at::Tensor> v;
      for (auto t : q.cast<py::list>()) v.push_back(t.cast<at::Tensor>());
      pub_.push_back(std::move(v));
    }
    pub_chunk_ = c["pub_chunk"].cast<int64_t>();
    pub_dtype_ = dtype_of(c["pub_dtype"].cast<int>());
    numel_ = master_.numel();
    ring_chunk_ = c["ring_chunk"].cast<int64_t>();
    for (auto r : c["rings"].cast<py::list>()) {
      std::vector<at::Tensor> v;
      if (!r.is_none())
        for (auto t : r.cast<py::list>()) v.push_back(t.cast<at::Tensor>());
      rings_.push_back(std::move(v));
    }
    for (auto r : c["remote"].cast<py::list>()) remote_.push_back(r.cast<bool>());
    for (auto o : c["buckets"].cast<py::list>()) {
      auto d = o.cast<py::dict>();
      BucketDesc b;
      b.lo = d["lo"].cast<int64_t>();
      b.hi = d["hi"].cast<int64_t>();
      b.msg_ext = d["msg_ext"].cast<int64_t>();
      b.wire_off = d["wire_off"].cast<int64_t>();
      b.msg_nbytes = d["msg_nbytes"].cast<int64_t>();
      b.kind = d["kind"].cast<int>();
      for (auto f : d["fields"].cast<py::list>()) {
        auto t = f.cast<py::tuple>();
        b.f.push_back(MsgField{t[0].cast<int64_t>(), t[1].cast<int64_t>(), dtype_of(t[2].cast<int>())});
      }
      buckets_.push_back(std::move(b));
    }
    for (auto o : c["groups"].cast<py::list>()) {
      auto d = o.cast<py::dict>();
      Group g{};
      g.a = d["a"].cast<int64_t>();
      g.b = d["b"].cast<int64_t>();
      g.adam = d["adam"].cast<bool>();
      g.steps = d["steps"].cast<int64_t>();
      groups_.push_back(g);
    }
    auto opt_t = [&](const char* k) { return c.contains(k) && !c[k].is_none() ? c[k].cast<at::Tensor>() : at::Tensor(); };
    mom_buf_ = opt_t("momentum_buffer");
    exp_avg_ = opt_t("exp_avg");
    exp_avg_sq_ = opt_t("exp_avg_sq");
    max_exp_avg_sq_ = opt_t("max_exp_avg_sq");
    csteps_ = opt_t("csteps");
    chunk_slots_ = opt_t("chunk_slots");
    // rehearsal: E emulated remote workers' PS load (PSConfig.emulate_remote)
    emu_ = c.contains("emu") ? c["emu"].cast<int>() : 0;
    if (emu_ > 0) {
      emu_in_ = c["emu_in"].cast<at::Tensor>();
      emu_sink_ = c["emu_sink"].cast<at::Tensor>();
      emu_stream_ = c["emu_stream"].cast<int64_t>();
      emu_traffic_ = c.contains("emu_traffic") ? c["emu_traffic"].cast<bool>() : true;
      hip_ok(hipEventCreateWithFlags(&emu_ev_, hipEventDisableTiming), "hipEventCreate");
    }
    if ((int)rings_.size() != W_ || (int)remote_.size() != W_) throw std::runtime_error("native PS: rings per worker");
    if ((int)buckets_.size() != nb_) throw std::runtime_error("native PS: bucket table");
    seen_.assign(W_, 0);
    dropping_.assign(W_, false);
    scale_.assign(W_, 1.0);
    count_b_.assign(nb_, 0);
    ver_b_.assign(nb_, 0);
    pending_b_.assign(nb_, {});
    incl_b_.assign(W_, std::vector<int64_t>(nb_, 0));
    pres_full_b_.assign(nb_, false);
    pres_part_b_.assign(nb_, at::Tensor());
    direct_.assign(nb_, Direct{});
  }
  ~NativePS() {  // never left running: an engine dropped without close() stops its loop here
    quit_ = true;
    if (th_.joinable()) {
      py::gil_scoped_release nogil;
      th_.join();
    }
    if (emu_ev_) hipEventDestroy(emu_ev_);
  }

  // hyper-parameters of group gi (pushed by Python at every step(): schedulers may change lr)
  void set_group(int gi, double lr, double wd, double mom, double damp, bool nesterov, double beta1, double beta2,
                 double eps, bool amsgrad, bool torch_mode) {
    std::lock_guard<std::mutex> lk(hp_mu_);
    Group& g = groups_.at(gi);
    g.lr = lr;
    g.wd = wd;
    g.mom = mom;
    g.damp = damp;
    g.nesterov = nesterov;
    g.beta1 = beta1;
    g.beta2 = beta2;
    g.eps = eps;
    g.amsgrad = amsgrad;
    g.torch_mode = torch_mode;
    hp_set_ = true;
  }

  void start() {
    if (th_.joinable()) throw std::runtime_error("native PS already started");
    if (!hp_set_) throw std::runtime_error("native PS: set the group hyper-parameters before start()");
    done_ = false;
    th_ = std::thread([this] { run(); });
  }
  // true once the loop has exited (timeout_s < 0: wait forever)
  bool join(double timeout_s) {
    if (!th_.joinable()) return true;
    {
      py::gil_scoped_release nogil;
      const auto t0 = std::chrono::steady_clock::now();
      while (!done_.load()) {
        if (timeout_s >= 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
          return false;
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
      }
      th_.join();
    }
    return true;
  }
  bool alive() const { return th_.joinable() && !done_.load(); }
  void pause(bool on) { pause_req_ = on; }
  bool paused() const { return paused_.load(); }
  bool pause_requested() const { return pause_req_.load(); }
  std::string error() {
    std::lock_guard<std::mutex> lk(err_mu_);
    return err_;
  }

  // counters (read between messages: under pause(), or after join())
  py::dict state() {
    py::dict d;
    std::lock_guard<std::mutex> lk(st_mu_);
    d["ver"] = ver_;
    d["seen"] = seen_;
    d["count_b"] = count_b_;
    d["ver_b"] = ver_b_;
    d["gsteps"] = gsteps_;
    std::vector<int64_t> gs;
    for (auto& g : groups_) gs.push_back(g.steps);
    d["group_steps"] = gs;
    py::dict s;
    for (auto& kv : stats_) s[py::str(kv.first)] = kv.second;
    d["stats"] = s;
    d["left_behind"] = left_behind_;
    return d;
  }
  // restore (load_engine_state, under pause() before training)
  void restore(int64_t ver, std::vector<int64_t> ver_b, std::vector<int64_t> count_b, int64_t gsteps,
               std::vector<int64_t> group_steps) {
    std::lock_guard<std::mutex> lk(st_mu_);
    ver_ = ver;
    if ((int)ver_b.size() == nb_) ver_b_ = ver_b;
    if ((int)count_b.size() == nb_) count_b_ = count_b;
    gsteps_ = gsteps;
    for (size_t i = 0; i < group_steps.size() && i < groups_.size(); ++i) groups_[i].steps = group_steps[i];
  }

 private:
  struct Direct {
    bool set = false;
    int64_t off = 0;
    int worker = 0;
    int64_t seq = 0;
    double scale = 1.0;
  };

  // bytes [off, off + n) of a worker's ring (a message never straddles two ring chunks)
  at::Tensor ring_bytes(int worker, int64_t off, int64_t n) const {
    const int64_t c = off / ring_chunk_, o = off - c * ring_chunk_;
    return rings_[worker].at(c).narrow(0, o, n);
  }
  at::Tensor view(int worker, int64_t off, const MsgField& f) const {
    return ring_bytes(worker, off + f.off, f.numel * (int64_t)c10::elementSize(f.dtype)).view(f.dtype);
  }
  // elements [a, b) of publish buffer k, inside one chunk
  at::Tensor pub_view(int k, int64_t a, int64_t b) const {
    const int64_t c = a / pub_chunk_;
    return pub_[k].at(c).narrow(0, a - c * pub_chunk_, b - a);
  }
  template <typename F>
  void pub_pieces(int64_t lo, int64_t hi, F fn) const {
    for (int64_t a = lo; a < hi;) {
      const int64_t b = std::min(hi, (a / pub_chunk_ + 1) * pub_chunk_);
      fn(a, b);
      a = b;
    }
  }
  void bump(const char* k, int64_t v = 1) { stats_[k] += v; }

  void run() {
    try {
      hipSetDevice(device_);
      c10::hip::HIPStream st = c10::hip::getStreamFromExternal(reinterpret_cast<hipStream_t>(stream_), device_);
      c10::hip::HIPStreamGuard sg(st);
      for (;;) {
        std::vector<int> ready = ctl_.wait_any_raw(seen_, 20000);
        {
          std::lock_guard<std::mutex> lk(st_mu_);
          for (int i : ready) pump(i);
          flush();
        }
        if (pause_req_.load()) hold();
        if (quit_.load() || should_stop()) break;
      }
      hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream_));
    } catch (const std::exception& e) {
      {
        std::lock_guard<std::mutex> lk(err_mu_);
        err_ = std::string("native PS loop: ") + e.what();
      }
      ctl_.store(ERROR, 0, 1);
      done_ = true;
      return;
    }
    // the PS leaves while a worker has not said STOP: that worker's next wait fails (ERROR = 2)
    for (int i = 0; i < W_; ++i)
      if (i != rank_ && ctl_.load(STOP, i) == 0) left_behind_.push_back(i);
    if (!left_behind_.empty()) ctl_.store(ERROR, 0, 2);
    done_ = true;
  }

  void hold() {
    hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream_));
    paused_ = true;
    while (pause_req_.load() && !ctl_.load(PS_STOP, 0) && !quit_.load()) {
      ctl_.ps_beat();
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    paused_ = false;
  }

  std::vector<int> dead_workers() {
    std::vector<int> out;
    const int64_t now = now_ns(), lim = dead_after_us_ * 1000;
    for (int i = 0; i < W_; ++i) {
      if (i == rank_) continue;  // the PS's own process is alive by construction
      const int64_t hb = ctl_.load(HEARTBEAT, i);
      if (hb && ctl_.load(STOP, i) == 0 && now - hb > lim) out.push_back(i);
    }
    return out;
  }

  bool should_stop() {
    if (ctl_.load(PS_STOP, 0)) return true;
    std::vector<int> dead = dead_workers();
    for (int i = 0; i < W_; ++i) {
      if (i != rank_ && std::find(dead.begin(), dead.end(), i) != dead.end()) continue;
      const int64_t stop = ctl_.load(STOP, i);
      if (stop == 0 || seen_[i] < stop - 1) return false;
    }
    return true;
  }

  void pump(int i) {
    const int64_t s_now = ctl_.load(PUSH_SEQ, i);
    for (int64_t s = seen_[i] + 1; s <= s_now; ++s) one(i, s);
    seen_[i] = std::max(seen_[i], s_now);
  }

  // ps_core.PSCore._one + _one_bucket (bucket granularity)
  void one(int i, int64_t s) {
    const int slot = (int)(s % SLOTS_);
    const int64_t pos = (s - 1) % nb_;
    const int vidx = i * MAXSLOTS_ + slot;
    const int64_t flag = ctl_.load(PUSH_FLAG, vidx);
    const int bi = (int)((flag >> 1) & ((1 << 20) - 1));
    const int64_t off = (flag >> 21) << 8;
    if (bi < 0 || bi >= nb_) throw std::runtime_error("message names an unknown bucket");
    if (pos == 0) {
      const int64_t pv = ctl_.load(PUSH_VER, vidx);
      const int64_t stale = ver_ - pv;
      dropping_[i] = staleness_ >= 0 && stale > staleness_;
      scale_[i] = staleness_lr_ ? 1.0 / (double)std::max<int64_t>(1, stale) : 1.0;
      if (!dropping_[i]) bump("staleness_sum", std::max<int64_t>(0, stale));
      ctl_.store(LAST_STALE, i, stale);
      ctl_.store(LAST_STALE_SEQ, i, s + nb_ - 1);
    }
    const int64_t step = (s - 1) / nb_ + 1;
    const bool kept = !dropping_[i];
    if (kept) {
      accumulate(i, off, bi, s, scale_[i]);
      note_presence(i, off, bi, flag);
    }
    ack(i, s);
    pending_b_[bi].push_back({i, step});
    if (pos == nb_ - 1) {
      if (kept) {
        bump("accumulated");
      } else {
        bump("drops");
        ctl_.fetch_add(DROPS, 0, 1);
      }
    }
    if (!kept) return;
    if (++count_b_[bi] < M_) return;
    ver_b_[bi] += 1;
    count_b_[bi] = 0;
    std::vector<int> touched;
    for (auto& ws : pending_b_[bi]) {
      if (ws.second > incl_b_[ws.first][bi]) incl_b_[ws.first][bi] = ws.second;
      if (std::find(touched.begin(), touched.end(), ws.first) == touched.end()) touched.push_back(ws.first);
    }
    pending_b_[bi].clear();
    std::vector<std::pair<int, int64_t>> incl;
    for (int w : touched)
      incl.push_back({w, *std::min_element(incl_b_[w].begin(), incl_b_[w].end()) * (int64_t)nb_});
    const int64_t gver = *std::min_element(ver_b_.begin(), ver_b_.end());
    const bool adv = gver > ver_;
    if (adv) ver_ = gver;
    flush();
    update_bucket(bi, ver_b_[bi], adv ? gver : -1, incl);
  }

  void accumulate(int i, int64_t off, int bi, int64_t seq, double scale) {
    const BucketDesc& b = buckets_[bi];
    if (direct_ok_ && !remote_[i] && b.kind == kDense) {
      // M = 1: the update reads the message itself; its slot is acked after that update
      direct_[bi] = Direct{true, off, i, seq, scale};
      return;
    }
    pend_.push_back(Pend{bi, scale, i, off, false});
    for (int e = 0; e < emu_; ++e) pend_.push_back(Pend{bi, scale, i, off, true});
  }

  void ack(int i, int64_t s) {
    for (auto& d : direct_)
      if (d.set && d.worker == i && d.seq == s) return;  // rung by update_bucket
    pend_acks_.push_back({i, s});
  }

  void note_presence(int i, int64_t off, int bi, int64_t flag) {
    if (!skip_missing_ || pres_full_b_[bi]) return;
    if (!(flag & 1)) {
      pres_full_b_[bi] = true;
      pres_part_b_[bi] = at::Tensor();
      return;
    }
    at::Tensor p = ring_bytes(i, off + buckets_[bi].msg_ext, ns_);
    if (remote_[i]) {
      at::Tensor t = at::empty({ns_}, p.options());
      copy_acquire(p, t);
      p = t;
    }
    at::Tensor& cur = pres_part_b_[bi];
    cur = cur.defined() ? at::maximum(cur, p) : p.clone();
  }

  void decode_into(const std::vector<const Pend*>& msgs, const BucketDesc& b, at::Tensor acc, double scale,
                   bool acquire) {
    auto V = [&](const Pend* m, int k) { return view(m->worker, m->off, b.f[k]); };
    switch (b.kind) {
      case kDense: {
        std::vector<at::Tensor> xs;
        for (auto* m : msgs) xs.push_back(V(m, 0));
        aggregate(xs, acc, scale, true, acquire);
        break;
      }
      case kQ8: {  // fields: q, scales
        std::vector<at::Tensor> qs, ss;
        for (auto* m : msgs) {
          qs.push_back(V(m, 0));
          ss.push_back(V(m, 1));
        }
        q8_aggregate(qs, ss, acc, scale, true, acquire);
        break;
      }
      case kTopk:  // idx, val
        for (auto* m : msgs) topk_accumulate(V(m, 0), V(m, 1), acc, scale, acquire);
        break;
      case kTopkQ8:  // idx, q, scales
        for (auto* m : msgs) topk_q8_accumulate(V(m, 0), V(m, 1), V(m, 2), acc, scale, acquire);
        break;
      case kThresh:  // count, idx, val
        for (auto* m : msgs) thresh_accumulate(V(m, 0), V(m, 1), V(m, 2), acc, scale, acquire);
        break;
      default:
        throw std::runtime_error("native PS: codec kind");
    }
  }

  // the messages that arrived together for one (bucket, scale), summed by one multi-source launch
  // per 16 (ps_async.PSAsyncEngine.flush), then the acks in order, 6 words per doorbell
  void flush() {
    if (!pend_.empty()) {
      // (an emulated remote copy joins its real message's batch: lockstep workers' messages for
      // a bucket arrive together)
      std::vector<std::pair<std::pair<int, double>, std::vector<const Pend*>>> groups;
      for (const Pend& p : pend_) {
        auto key = std::make_pair(p.bi, p.scale);
        auto it = std::find_if(groups.begin(), groups.end(), [&](auto& g) { return g.first == key; });
        if (it == groups.end()) {
          groups.push_back({key, {}});
          it = groups.end() - 1;
        }
        it->second.push_back(&p);
      }
      for (auto& g : groups) {
        const BucketDesc& b = buckets_[g.first.first];
        at::Tensor acc = acc_.narrow(0, acc_scratch_ ? 0 : b.lo, b.hi - b.lo);
        auto& ms = g.second;
        for (size_t k = 0; k < ms.size(); k += 16) {
          std::vector<const Pend*> part(ms.begin() + k, ms.begin() + std::min(ms.size(), k + 16));
          bool acq = false;
          for (auto* m : part) acq |= remote_[m->worker];
          decode_into(part, b, acc, g.first.second, acq);
          bump("acc_launches");
        }
      }
      pend_.clear();
    }
    for (size_t k = 0; k < pend_acks_.size(); k += 6) {
      std::vector<std::tuple<int, int, int64_t>> w;
      for (size_t j = k; j < std::min(pend_acks_.size(), k + 6); ++j)
        w.emplace_back(ACK_SEQ, pend_acks_[j].first, pend_acks_[j].second);
      ctl_.enqueue(stream_, w);
    }
    pend_acks_.clear();
  }

  // optimizer step of flat [lo, hi) (inside one publish chunk) publishing into buffer k
  void update_range(const at::Tensor& src, int64_t src_lo, int64_t lo, int64_t hi, double gscale, bool zero_src,
                    int k, const at::Tensor& mask) {
    std::lock_guard<std::mutex> lk(hp_mu_);
    for (Group& g : groups_) {
      const int64_t a = std::max(g.a, lo), b = std::min(g.b, hi);
      if (b <= a) continue;
      std::vector<at::Tensor> srcs{src.narrow(0, a - src_lo, b - a)};
      at::Tensor tgt = master_.narrow(0, a, b - a);
      c10::optional<at::Tensor> pb = pub_view(k, a, b);
      c10::optional<at::Tensor> mk;
      if (mask.defined()) mk = mask.narrow(0, a / 16, (b - a) / 16);
      c10::optional<at::Tensor> cs;
      if (csteps_.defined()) cs = csteps_.narrow(0, a / 16, (b - a) / 16);
      if (!g.adam) {
        c10::optional<at::Tensor> buf;
        if (g.mom != 0.0) {
          if (!mom_buf_.defined()) throw std::runtime_error("native PS: momentum buffer missing");
          buf = mom_buf_.narrow(0, a, b - a);
        } else {
          cs = c10::nullopt;
        }
        sgd_step(srcs, gscale, tgt, buf, pb, zero_src, g.lr, g.wd, g.mom, g.damp, g.nesterov, false, mk, cs, 0.0);
      } else {
        c10::optional<at::Tensor> vm;
        if (g.amsgrad) vm = max_exp_avg_sq_.narrow(0, a, b - a);
        adam_step(srcs, gscale, tgt, exp_avg_.narrow(0, a, b - a), exp_avg_sq_.narrow(0, a, b - a), vm, pb, zero_src,
                  g.lr, g.beta1, g.beta2, g.eps, g.wd, g.steps, g.amsgrad, g.torch_mode, mk, cs);
      }
    }
  }

  // PSAsyncEngine.update_bucket
  void update_bucket(int bi, int64_t v, int64_t gver, const std::vector<std::pair<int, int64_t>>& incl) {
    const BucketDesc& b = buckets_[bi];
    const int k = (int)(v % npub_);
    const int idx = bi * npub_ + k;
    const int64_t old = ctl_.load(BBUF_VER, idx);
    ctl_.store(BBUF_VER, idx, -1);  // readers skip a slot being rewritten ...
    if (old >= 0 && !ctl_.wait_no_reader_b_raw(bi, old, 0)) {  // ... and it waits for current readers
      bump("reader_waits");
      if (!ctl_.wait_no_reader_b_raw(bi, old, dead_after_us_)) bump("reader_timeouts");
    }
    at::Tensor mask;
    if (skip_missing_ && !pres_full_b_[bi] && pres_part_b_[bi].defined()) {
      if (!chunk_slots_.defined()) throw std::runtime_error("native PS: chunk table missing");
      mask = pres_part_b_[bi].index_select(0, chunk_slots_);
    }
    pres_full_b_[bi] = false;
    pres_part_b_[bi] = at::Tensor();
    const int64_t top = *std::max_element(ver_b_.begin(), ver_b_.end());
    if (top > gsteps_) {  // group step hint (per-chunk counts decide the optimizer math)
      std::lock_guard<std::mutex> lk(hp_mu_);
      for (Group& g : groups_)
        if (g.b > g.a) g.steps += 1;
      gsteps_ = top;
    }
    Direct d = direct_[bi];
    direct_[bi] = Direct{};
    if (d.set) {  // straight from the mailbox slot (M = 1)
      at::Tensor msg = view(d.worker, d.off, b.f[0]);
      pub_pieces(b.lo, b.hi, [&](int64_t pa, int64_t pb) {
        update_range(msg, b.lo, pa, pb, gscale_ * d.scale, false, k, mask);
      });
      bump("direct_updates");
    } else {
      pub_pieces(b.lo, b.hi, [&](int64_t pa, int64_t pb) {
        update_range(acc_, acc_scratch_ ? b.lo : 0, pa, pb, gscale_, true, k, mask);
      });
    }
    std::vector<std::tuple<int, int, int64_t>> words;
    if (d.set) words.emplace_back(ACK_SEQ, d.worker, d.seq);  // the slot is free once the update read it
    words.emplace_back(BBUF_VER, idx, v);
    words.emplace_back(BPUB_VER, bi, v);
    if (gver >= 0) words.emplace_back(PUB_VER, 0, gver);
    for (auto& wi : incl) words.emplace_back(INCL_SEQ, wi.first, wi.second);
    for (size_t j = 0; j < words.size(); j += 6)
      ctl_.enqueue(stream_, std::vector<std::tuple<int, int, int64_t>>(
                                words.begin() + j, words.begin() + std::min(words.size(), j + 6)));
    if (emu_ > 0 && emu_traffic_) emulate_traffic(k, bi);
    if (gver >= 0) ctl_.fetch_add(UPDATES, 0, 1);
    bump("bucket_updates");
  }

  // PSAsyncEngine._emulate_remote_traffic: E write sweeps of the bucket's message bytes (their
  // pushes landing) and E read sweeps of its publish range (their pulls), on a low-priority stream
  // ordered after the update
  void emulate_traffic(int k, int bi) {
    const BucketDesc& b = buckets_[bi];
    hipStream_t ps = reinterpret_cast<hipStream_t>(stream_), es = reinterpret_cast<hipStream_t>(emu_stream_);
    if (es != ps) {
      hip_ok(hipEventRecord(emu_ev_, ps), "hipEventRecord");
      hip_ok(hipStreamWaitEvent(es, emu_ev_, 0), "hipStreamWaitEvent");
    }
    c10::hip::HIPStreamGuard g(c10::hip::getStreamFromExternal(es, device_));
    at::Tensor win = emu_in_.narrow(0, b.wire_off, b.msg_nbytes);
    for (int e = 0; e < emu_; ++e) {  // (few workgroups: see rt::emu_sweep)
      bool first = true;
      pub_pieces(b.lo, b.hi, [&](int64_t pa, int64_t pb) {
        emu_sweep(first ? win : win.narrow(0, 0, 0), pub_view(k, pa, pb), emu_sink_, e + 1, 8);
        first = false;
      });
    }
  }
  static void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
  }

  ControlBlock& ctl_;
  int W_, rank_, nb_, SLOTS_, MAXSLOTS_, M_, npub_, device_;
  int64_t staleness_, dead_after_us_, ns_, stream_, numel_;
  bool staleness_lr_, skip_missing_, direct_ok_, acc_scratch_ = false;
  double gscale_;
  at::Tensor acc_, master_, mom_buf_, exp_avg_, exp_avg_sq_, max_exp_avg_sq_, csteps_, chunk_slots_;
  std::vector<std::vector<at::Tensor>> pub_;  // [npub][chunk]
  int64_t pub_chunk_ = 0, ring_chunk_ = 0;
  at::ScalarType pub_dtype_;
  int emu_ = 0;
  bool emu_traffic_ = true;
  int64_t emu_stream_ = 0;
  hipEvent_t emu_ev_ = nullptr;
  at::Tensor emu_in_, emu_sink_;
  std::vector<std::vector<at::Tensor>> rings_;  // [worker][chunk] (uint8)
  std::vector<bool> remote_;
  std::vector<BucketDesc> buckets_;
  std::vector<Group> groups_;
  std::mutex hp_mu_, st_mu_, err_mu_;
  bool hp_set_ = false;

  // protocol state (ps_core.PSCore, bucket granularity)
  int64_t ver_ = 0, gsteps_ = 0;
  std::vector<int64_t> seen_, count_b_, ver_b_;
  std::vector<bool> dropping_, pres_full_b_;
  std::vector<double> scale_;
  std::vector<std::vector<std::pair<int, int64_t>>> pending_b_;
  std::vector<std::vector<int64_t>> incl_b_;
  std::vector<at::Tensor> pres_part_b_;
  std::vector<Pend> pend_;
  std::vector<std::pair<int, int64_t>> pend_acks_;
  std::vector<Direct> direct_;
  std::map<std::string, int64_t> stats_;
  std::vector<int> left_behind_;

  std::thread th_;
  std::atomic<bool> done_{true}, pause_req_{false}, paused_{false}, quit_{false};
  std::string err_;
};

void bind_psloop(py::module& m) {
  py::class_<NativePS>(m, "NativePS")
      .def(py::init<ControlBlock&, py::dict>(), py::arg("ctl"), py::arg("cfg"), py::keep_alive<1, 2>())
      .def("set_group", &NativePS::set_group)
      .def("start", &NativePS::start)
      .def("join", &NativePS::join, py::arg("timeout_s") = -1.0)
      .def("alive", &NativePS::alive)
      .def("pause", &NativePS::pause)
      .def("paused", &NativePS::paused)
      .def("pause_requested", &NativePS::pause_requested)
      .def("error", &NativePS::error)
      .def("state", &NativePS::state)
      .def("restore", &NativePS::restore);
}

}  // namespace rt
}  // namespace hipps
