#include "ps.h"
#include "trace.h"

#include <xmmintrin.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "../kernels/kernels.h"

namespace mpit {

namespace {
void hipp(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("mpit ps HIP error in ") + what + ": " + hipGetErrorString(e));
}
}  // namespace

// =========================================================================== server

PSServer::PSServer(Engine& eng, int ps_id, Window& rx, Window& tx, std::vector<int> members, std::vector<int> clients,
                   int64_t shard_off, int64_t shard_len, bool device, uintptr_t p, std::vector<uintptr_t> state,
                   uintptr_t inbox, ServerRule rule, int datapath, int64_t staleness, bool grad_bf16, int init_rank)
    : eng_(eng),
      ps_id_(ps_id),
      rx_(rx),
      tx_(tx),
      members_(std::move(members)),
      clients_(std::move(clients)),
      off_(shard_off),
      len_(shard_len),
      device_(device),
      p_(reinterpret_cast<void*>(p)),
      inbox_(reinterpret_cast<void*>(inbox)),
      rule_(rule),
      lr_(rule.lr),
      datapath_(datapath),
      staleness_(staleness),
      grad_bf16_(grad_bf16),
      init_rank_(init_rank) {
  for (auto s : state) st_.push_back(reinterpret_cast<void*>(s));
  static const int need[] = {0, 3, 2, 2, 1, 2};
  if (rule_.kind < 0 || rule_.kind > 5) throw std::invalid_argument("mpit: unknown server rule");
  if (int(st_.size()) < need[rule_.kind]) throw std::invalid_argument("mpit: missing server optimizer state buffers");
  if (device_ && eng_.device() < 0) throw std::invalid_argument("mpit: device server on a rank without a device");
  if (device_ && datapath_ == 1 && !inbox_) throw std::invalid_argument("mpit: datapath 1 needs an inbox buffer");
  clock_.assign(clients_.size(), 0);
  if (device_) {
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    int lo = 0, hi = 0;
    hipp(hipDeviceGetStreamPriorityRange(&lo, &hi), "priority range");
    hipp(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "server stream");
    if (datapath_ == 2) {
      const size_t nc = clients_.size();
      cstream_.resize(nc);
      ev_in_.resize(nc);
      ev_up_.resize(nc);
      ev_out_.resize(nc);
      for (size_t i = 0; i < nc; ++i) {
        hipp(hipStreamCreateWithPriority(&cstream_[i], hipStreamNonBlocking, hi), "link stream");
        hipp(hipEventCreateWithFlags(&ev_in_[i], hipEventDisableTiming), "event");
        hipp(hipEventCreateWithFlags(&ev_up_[i], hipEventDisableTiming), "event");
        hipp(hipEventCreateWithFlags(&ev_out_[i], hipEventDisableTiming), "event");
      }
      if (nc && len_ > 0) hipp(hipMalloc(reinterpret_cast<void**>(&stage_), nc * size_t(len_) * 8), "hipMalloc(stage)");
    }
  }
}

PSServer::~PSServer() {
  for (int t = 1; t <= 8; ++t) eng_.register_am(ps_am_id(ps_id_, t), [](const Msg&) {});
  if (stream_) {
    hipSetDevice(eng_.device());
    for (auto s : cstream_) {
      hipStreamSynchronize(s);
      hipStreamDestroy(s);
    }
    hipStreamSynchronize(stream_);
    hipStreamDestroy(stream_);
    for (auto* v : {&ev_in_, &ev_up_, &ev_out_})
      for (auto e : *v) hipEventDestroy(e);
    if (stage_) hipFree(stage_);
  }
}

void PSServer::finish_on(hipStream_t s, std::function<void()> then) {
  hipEvent_t ev;
  hipp(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
  hipp(hipEventRecord(ev, s), "hipEventRecord");
  eng_.track_copy(ev, std::move(then));
}

void PSServer::start() {
  for (int t : {kTagInit, kTagGrad, kTagParam, kTagHeader, kTagStop})
    eng_.register_am(ps_am_id(ps_id_, t), [this](const Msg& m) { on_msg(m); });
}

int PSServer::member_of(int world_rank) const {
  for (size_t i = 0; i < members_.size(); ++i)
    if (members_[i] == world_rank) return int(i);
  throw std::invalid_argument("mpit: PS message from a rank outside the window group");
}

int PSServer::client_index(int world_rank) const {
  for (size_t i = 0; i < clients_.size(); ++i)
    if (clients_[i] == world_rank) return int(i);
  return -1;
}

void PSServer::on_msg(const Msg& m) {
  const int tag = (m.tag - 4096) % 16;
  // asyncsgd/pserver.lua:152-158: the shard is initialised from the first client's
  // parameter push before any gradient or pull is served
  if (init_rank_ >= 0 && (tag == kTagGrad || tag == kTagHeader)) {
    backlog_.push_back(m);
    return;
  }
  switch (tag) {
    case kTagInit:
      if (m.aux0 != off_ || m.aux1 != len_)
        std::fprintf(stderr, "[mpit ps %d] client %d shard (%lld,%lld) != server shard (%lld,%lld)\n", ps_id_, m.src,
                     (long long)m.aux0, (long long)m.aux1, (long long)off_, (long long)len_);
      break;
    case kTagParam:
      do_param(m.src, (m.aux0 & kPsFromRx) != 0);
      if (init_rank_ >= 0 && m.src == init_rank_) {
        init_rank_ = -1;
        std::vector<Msg> later;
        later.swap(backlog_);
        for (auto& x : later) on_msg(x);
      }
      break;
    case kTagGrad: do_grad(m.src, (m.aux0 & kPsWithPull) != 0); break;
    case kTagHeader: {
      const int ci = client_index(m.src);
      if (staleness_ >= 0 && ci >= 0) {
        int64_t mn = clock_[0];
        for (auto c : clock_) mn = std::min(mn, c);
        if (clock_[size_t(ci)] - mn > staleness_) {
          std::lock_guard<std::mutex> g(mu_);
          deferred_.push_back(m.src);
          ++stats_.deferred;
          break;
        }
      }
      do_pull(m.src);
      break;
    }
    case kTagStop: {
      stopped_.fetch_add(1);
      // a stopped client no longer holds back the stragglers' clocks
      const int ci = client_index(m.src);
      if (ci >= 0) clock_[size_t(ci)] = INT64_MAX / 4;
      release_deferred();
      std::lock_guard<std::mutex> g(mu_);
      cv_.notify_all();
      break;
    }
    default:
      std::fprintf(stderr, "[mpit ps %d] unexpected tag %d from %d\n", ps_id_, tag, m.src);
  }
}

void PSServer::finish(std::function<void()> then) {
  if (!device_) {
    then();
    return;
  }
  hipEvent_t ev;
  hipp(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
  hipp(hipEventRecord(ev, stream_), "hipEventRecord");
  eng_.track_copy(ev, std::move(then));
}

void PSServer::reply(int c, int tag) { eng_.send_am(c, ps_am_id(ps_id_, tag), nullptr, 0); }

void PSServer::apply_rule(const void* g, void* out) {
  const int dev = device_ ? eng_.device() : -1;
  const uint32_t bf = grad_bf16_ ? 2u : 0u;
  const int v = out ? kOut : 0;
  auto P = [](const void* x) { return reinterpret_cast<uintptr_t>(x); };
  std::vector<uintptr_t> ptrs{P(p_), P(g)};
  for (size_t k = 0; k < st_.size(); ++k) {
    static const int need[] = {0, 3, 2, 2, 1, 2};
    if (int(k) < need[rule_.kind]) ptrs.push_back(P(st_[k]));
  }
  if (out) ptrs.push_back(P(out));
  ServerRule r = rule_;  // progress thread only; lr may be changed concurrently (set_lr)
  r.lr = lr_.load(std::memory_order_relaxed);
  switch (r.kind) {
    case 0:
      ew_update(kApply, v, dev, stream_, len_, ptrs, bf, {r.a});
      break;
    case 1:
      ew_update(kRMSProp, v | kAdd, dev, stream_, len_, ptrs, bf, {r.decay, r.lr, r.mom, r.eps});
      break;
    case 2: {  // BiCNN/pserver.lua:147-154: bias correction on floor(t/stepDiv)+1
      ++t_;
      const double k = double(t_.load() / std::max<int64_t>(1, r.step_div) + 1);
      const double lr_t = r.lr * std::sqrt(1.0 - std::pow(double(r.b2), k)) / (1.0 - std::pow(double(r.b1), k));
      ew_update(kAdam, v, dev, stream_, len_, ptrs, bf, {r.b1, r.b2, r.eps, float(lr_t)});
      break;
    }
    case 3: {  // BiCNN/pserver.lua:163-170
      ++t_;
      const double lr_t = r.lr / (1.0 - std::pow(double(r.b1), double(t_.load())));
      ew_update(kAdamax, v, dev, stream_, len_, ptrs, bf, {r.b1, r.b2, r.eps, float(lr_t)});
      break;
    }
    case 4: {  // BiCNN/pserver.lua:177-182
      const float clr = float(r.lr / (1.0 + double(t_.load()) * r.lrd));
      ++t_;
      ew_update(kAdagrad, v, dev, stream_, len_, ptrs, bf, {r.eps, clr});
      break;
    }
    case 5:  // BiCNN/pserver.lua:189-193
      ++t_;
      ew_update(kAdadelta, v, dev, stream_, len_, ptrs, bf, {r.rho, r.eps, r.lr});
      break;
  }
  version_.fetch_add(1);
}

void PSServer::do_param(int c, bool from_rx) {
  TraceRange tr("ps_server_param");
  const int m = member_of(c);
  const Window& w = from_rx ? rx_ : tx_;  // rx is always fp32
  const bool bf = grad_bf16_ && !from_rx;
  const int64_t es = bf ? 2 : 4;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(w.remote_ptr(m)) + off_ * es;
  if (!device_ && w.remote_device(m)) throw std::runtime_error("mpit: host server cannot read a device window");
  if (device_) hipp(hipSetDevice(eng_.device()), "hipSetDevice");
  // p (fp32) = pushed shard (fp32 | bf16): one copy / cast kernel, or a host loop
  ew_update(kCopy, 0, device_ ? eng_.device() : -1, stream_, len_,
            {reinterpret_cast<uintptr_t>(p_), reinterpret_cast<uintptr_t>(src)}, bf ? 2u : 0u, {1.f});
  {
    std::lock_guard<std::mutex> g(mu_);
    ++stats_.param_pushes;
  }
  finish([this, c] { reply(c, kTagParamTail); });
}

void PSServer::copy_out(int c) {
  const int m = member_of(c);
  uint8_t* dst = reinterpret_cast<uint8_t*>(rx_.remote_ptr(m)) + off_ * 4;
  if (device_) {
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    if (datapath_ != 1)
      ew_update(kCopy, 0, eng_.device(), stream_, len_, {reinterpret_cast<uintptr_t>(dst), reinterpret_cast<uintptr_t>(p_)},
                0u, {1.f});
    else
      hipp(hipMemcpyAsync(dst, p_, size_t(len_) * 4, hipMemcpyDefault, stream_), "param pull copy");
  } else {
    if (rx_.remote_device(m)) throw std::runtime_error("mpit: host server cannot write a device rx window");
    std::memcpy(dst, p_, size_t(len_) * 4);
  }
}

void PSServer::do_pull(int c) {
  TraceRange tr("ps_server_pull");
  const int ci = client_index(c);
  if (pipelined(ci, c)) {
    // snapshot the shard in update order on stream_, push it over the client's link
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    hipStream_t cs = cstream_[size_t(ci)];
    uint8_t* out = stage_ + size_t(ci) * size_t(len_) * 8 + size_t(len_) * 4;
    uint8_t* dst = reinterpret_cast<uint8_t*>(rx_.remote_ptr(member_of(c))) + off_ * 4;
    hipp(hipStreamWaitEvent(stream_, ev_out_[size_t(ci)], 0), "wait outbox free");
    ew_update(kCopy, 0, eng_.device(), stream_, len_, {reinterpret_cast<uintptr_t>(out), reinterpret_cast<uintptr_t>(p_)},
              0u, {1.f});
    hipp(hipEventRecord(ev_up_[size_t(ci)], stream_), "record snapshot");
    hipp(hipStreamWaitEvent(cs, ev_up_[size_t(ci)], 0), "link waits snapshot");
    hipp(hipMemcpyAsync(dst, out, size_t(len_) * 4, hipMemcpyDefault, cs), "param push (link)");
    hipp(hipEventRecord(ev_out_[size_t(ci)], cs), "record outbox sent");
    {
      std::lock_guard<std::mutex> g(mu_);
      ++stats_.pulls;
    }
    finish_on(cs, [this, c] { reply(c, kTagSendParam); });
    return;
  }
  copy_out(c);
  {
    std::lock_guard<std::mutex> g(mu_);
    ++stats_.pulls;
  }
  finish([this, c] { reply(c, kTagSendParam); });
}

void PSServer::do_grad(int c, bool pull) {
  TraceRange tr(pull ? "ps_server_update+pull" : "ps_server_update");
  const int m = member_of(c);
  const int64_t es = grad_bf16_ ? 2 : 4;
  const void* g = reinterpret_cast<const uint8_t*>(tx_.remote_ptr(m)) + off_ * es;
  const int ci = client_index(c);
  bool defer_pull = false;
  if (ci >= 0) {
    ++clock_[size_t(ci)];
    if (pull && staleness_ >= 0) {
      int64_t mn = clock_[0];
      for (auto x : clock_) mn = std::min(mn, x);
      defer_pull = clock_[size_t(ci)] - mn > staleness_;
    }
  }
  if (!device_ && tx_.remote_device(m)) throw std::runtime_error("mpit: host server cannot read a device tx window");
  if (pipelined(ci, c)) {
    // link stream: pull the gradient shard into this client's inbox; stream_: fused update
    // (+ snapshot into the outbox when a pull is due); link stream: push the snapshot
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    const size_t k = size_t(ci);
    hipStream_t cs = cstream_[k];
    uint8_t* in = stage_ + k * size_t(len_) * 8;
    uint8_t* out = in + size_t(len_) * 4;
    const bool push_back = pull && !defer_pull;
    hipp(hipMemcpyAsync(in, g, size_t(len_ * es), hipMemcpyDefault, cs), "grad pull (link)");
    hipp(hipEventRecord(ev_in_[k], cs), "record inbox full");
    hipp(hipStreamWaitEvent(stream_, ev_in_[k], 0), "update waits inbox");
    if (push_back) hipp(hipStreamWaitEvent(stream_, ev_out_[k], 0), "update waits outbox free");
    apply_rule(in, push_back ? out : nullptr);
    hipp(hipEventRecord(ev_up_[k], stream_), "record update");
    hipp(hipStreamWaitEvent(cs, ev_up_[k], 0), "link waits update");  // inbox reusable after this
    if (push_back) {
      uint8_t* dst = reinterpret_cast<uint8_t*>(rx_.remote_ptr(m)) + off_ * 4;
      hipp(hipMemcpyAsync(dst, out, size_t(len_) * 4, hipMemcpyDefault, cs), "param push (link)");
      hipp(hipEventRecord(ev_out_[k], cs), "record outbox sent");
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      ++stats_.grads;
      if (push_back) ++stats_.pulls;
      if (defer_pull) {
        deferred_.push_back(c);
        ++stats_.deferred;
      }
    }
    finish_on(cs, [this, c, push_back] {
      reply(c, kTagGradTail);
      if (push_back) reply(c, kTagSendParam);
    });
    release_deferred();
    return;
  }
  void* fused_out = nullptr;
  if (pull && !defer_pull && (datapath_ != 1 || !device_))
    fused_out = reinterpret_cast<uint8_t*>(rx_.remote_ptr(m)) + off_ * 4;
  if (device_) {
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    if (datapath_ == 1) {
      hipp(hipMemcpyAsync(inbox_, g, size_t(len_ * es), hipMemcpyDefault, stream_), "grad inbox copy");
      g = inbox_;
    }
  }
  apply_rule(g, fused_out);
  if (pull && !defer_pull && !fused_out) copy_out(c);
  {
    std::lock_guard<std::mutex> lk(mu_);
    ++stats_.grads;
    if (pull && !defer_pull) ++stats_.pulls;
    if (defer_pull) {
      deferred_.push_back(c);
      ++stats_.deferred;
    }
  }
  finish([this, c, pull, defer_pull] {
    reply(c, kTagGradTail);
    if (pull && !defer_pull) reply(c, kTagSendParam);
  });
  release_deferred();
}

void PSServer::release_deferred() {
  if (staleness_ < 0) return;
  std::deque<int> ready;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (deferred_.empty()) return;
    int64_t mn = clock_.empty() ? 0 : clock_[0];
    for (auto x : clock_) mn = std::min(mn, x);
    std::deque<int> keep;
    for (int c : deferred_) {
      const int ci = client_index(c);
      if (ci < 0 || clock_[size_t(ci)] - mn <= staleness_) ready.push_back(c);
      else keep.push_back(c);
    }
    deferred_.swap(keep);
  }
  for (int c : ready) do_pull(c);
}

void PSServer::wait_done() {
  std::unique_lock<std::mutex> g(mu_);
  cv_.wait(g, [this] { return done(); });
}

ServerStats PSServer::stats() const {
  std::lock_guard<std::mutex> g(mu_);
  return stats_;
}

void PSServer::set_lr(float lr) { lr_.store(lr, std::memory_order_relaxed); }

void PSServer::sync() {
  if (device_) {
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    hipp(hipStreamSynchronize(stream_), "server sync");
  }
}

// =========================================================================== client

// One FIFO per client keeps the AMs of one client in call order even when they are
// gated on GPU work (a pull must never overtake the push issued before it).
struct PSClient::GateQueue {
  struct Gate {
    hipEvent_t ev;
    std::function<void()> send;
  };
  std::mutex mu;
  std::deque<Gate> q;
};

PSClient::PSClient(Engine& eng, int ps_id, std::vector<int> servers, std::vector<int64_t> offs,
                   std::vector<int64_t> lens)
    : eng_(eng), ps_id_(ps_id), servers_(std::move(servers)), offs_(std::move(offs)), lens_(std::move(lens)) {
  if (servers_.size() != offs_.size() || servers_.size() != lens_.size())
    throw std::invalid_argument("mpit: PSClient shard table mismatch");
  auto gq = std::make_shared<GateQueue>();
  gq_ = gq;
  int dev = eng_.device();
  hook_ = eng_.add_hook([gq, dev]() {
    bool did = false;
    for (;;) {
      GateQueue::Gate g;
      {
        std::lock_guard<std::mutex> l(gq->mu);
        if (gq->q.empty()) break;
        g = gq->q.front();
        if (g.ev) {
          hipSetDevice(dev);
          if (hipEventQuery(g.ev) == hipErrorNotReady) break;
        }
        gq->q.pop_front();
      }
      if (g.ev) hipEventDestroy(g.ev);
      g.send();
      did = true;
    }
    return did;
  });
}

PSClient::~PSClient() {
  if (hook_ >= 0) eng_.remove_hook(hook_);
}

void PSClient::start() {
  for (int t : {kTagSendParam, kTagParamTail, kTagGradTail})
    eng_.register_am(ps_am_id(ps_id_, t), [this](const Msg& m) { on_reply(m); });
  for (size_t i = 0; i < servers_.size(); ++i)
    eng_.send_am(servers_[i], ps_am_id(ps_id_, kTagInit), nullptr, 0, offs_[i], lens_[i]);
}

void PSClient::gate(hipStream_t s, std::function<void()> send) {
  GateQueue::Gate g{nullptr, std::move(send)};
  // s == 0 is the null stream (PyTorch's default stream on ROCm), not "no stream": a device
  // client always gates its AM on the work queued so far on s
  if (eng_.device() >= 0) {
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    hipp(hipEventCreateWithFlags(&g.ev, hipEventDisableTiming), "hipEventCreate");
    hipp(hipEventRecord(g.ev, s), "hipEventRecord");
  }
  std::lock_guard<std::mutex> l(gq_->mu);
  gq_->q.push_back(g);
}

void PSClient::send_grad(hipStream_t s, bool with_pull) {
  const int64_t n = int64_t(servers_.size());
  pending_.fetch_add(with_pull ? 2 * n : n);
  gate(s, [this, with_pull] {
    for (int srv : servers_) eng_.send_am(srv, ps_am_id(ps_id_, kTagGrad), nullptr, 0, with_pull ? kPsWithPull : 0);
  });
}

void PSClient::send_grad_to(hipStream_t s, int k, bool with_pull) {
  if (k < 0 || k >= int(servers_.size())) throw std::out_of_range("PSClient::send_grad_to: bad shard");
  pending_.fetch_add(with_pull ? 2 : 1);
  const int srv = servers_[k];
  gate(s, [this, srv, with_pull] {
    eng_.send_am(srv, ps_am_id(ps_id_, kTagGrad), nullptr, 0, with_pull ? kPsWithPull : 0);
  });
}

void PSClient::recv_param(hipStream_t s) {
  pending_.fetch_add(int64_t(servers_.size()));
  // ordered behind any gated push of this client
  gate(s, [this] {
    for (int srv : servers_) eng_.send_am(srv, ps_am_id(ps_id_, kTagHeader), nullptr, 0);
  });
}

void PSClient::send_param(hipStream_t s, bool from_rx) {
  pending_.fetch_add(int64_t(servers_.size()));
  gate(s, [this, from_rx] {
    for (int srv : servers_) eng_.send_am(srv, ps_am_id(ps_id_, kTagParam), nullptr, 0, from_rx ? kPsFromRx : 0);
  });
}

void PSClient::stop() {
  wait();
  for (int srv : servers_) eng_.send_am(srv, ps_am_id(ps_id_, kTagStop), nullptr, 0);
}

void PSClient::on_reply(const Msg&) {
  replies_.fetch_add(1);
  pending_.fetch_sub(1);
  pending_.notify_all();
}

// The worker waits here every step while the GPU finishes its backward (tens of ms).
// MPIT_WAIT_SPIN_US > 0 polls (pause) for up to that long before the futex sleep, keeping
// the core awake for the step start that follows (device clients only). Measured within
// noise of sleeping at once (profiles/step_start_host_r02.md): default 0.
void PSClient::wait() {
  static const int64_t spin_us = [] {
    const char* e = std::getenv("MPIT_WAIT_SPIN_US");
    return e ? std::max<int64_t>(0, std::atoll(e)) : int64_t(0);
  }();
  if (spin_us > 0 && eng_.device() >= 0) {  // GPU workers only (CPU ranks share few cores)
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0;; ++i) {
      if (pending_.load(std::memory_order_acquire) <= 0) return;
      _mm_pause();
      if ((i & 1023) == 0 &&
          std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us))
        break;
    }
  }
  for (;;) {
    const int64_t v = pending_.load(std::memory_order_acquire);
    if (v <= 0) return;
    pending_.wait(v, std::memory_order_acquire);
  }
}

}  // namespace mpit
