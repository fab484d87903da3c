#include "ps.h"
#include "trace.h"

#include <xmmintrin.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>

#include "../kernels/kernels.h"

namespace mpit {

// Co-located device clients (PSClient::local): a server on the same rank hands its update's
// GPU event to the client and replies at once. MPIT_PS_LOCAL_EVENTS=0: reply after a host
// poll of that event (the step boundary then pays the poll and the reply's wake-up while the
// GPU idles: the update kernel -> next step's weight cast gap, profiles/step_idle_r06.md).
namespace {
std::mutex g_local_mu;
std::map<std::pair<int, int>, PSClient*> g_local_clients;
std::map<std::pair<int, int>, PSServer*> g_local_servers;
bool local_events() {
  static const bool on = [] {
    const char* e = std::getenv("MPIT_PS_LOCAL_EVENTS");
    return !(e && e[0] == '0');
  }();
  return on;
}
// MPIT_PS_LOCAL_GATE=1 (A/B, off): the co-located client's messages also skip the host gate
// (PSClient::send_local). The step boundary's idle goes (0.6 -> 0.2 ms traced), but the host
// then queues a whole backward ahead of the GPU and the backward-weight side stream's small
// kernels end up behind the critical stream's (split_reduce 1.3 -> 3.9 ms per fp32 step):
// fp32 neutral, bf16 -6 % (gpurun_out/r06n, profiles/ps_local_events_r06.md)
bool local_gate() {
  static const bool on = [] {
    const char* e = std::getenv("MPIT_PS_LOCAL_GATE");
    return e && e[0] == '1';
  }();
  return on;
}
}  // namespace

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
      init_rank_(init_rank),
      init_left_(shard_len) {
  for (auto s : state) st_.push_back(reinterpret_cast<void*>(s));
  static const int need[] = {0, 3, 2, 2, 1, 2};
  if (rule_.kind < 0 || rule_.kind > 5) throw std::invalid_argument("mpit: unknown server rule");
  if (int(st_.size()) < need[rule_.kind]) throw std::invalid_argument("mpit: missing server optimizer state buffers");
  if (device_ && eng_.device() < 0) throw std::invalid_argument("mpit: device server on a rank without a device");
  if (device_ && datapath_ == 1 && !inbox_) throw std::invalid_argument("mpit: datapath 1 needs an inbox buffer");
  if (const char* e = std::getenv("MPIT_PS_FORCE_PIPE")) force_pipe_ = std::atoi(e) != 0;
  if (const char* e = std::getenv("MPIT_PS_BATCH")) batch_ = std::atoi(e) != 0;
  if (const char* e = std::getenv("MPIT_PS_FAULT")) {
    const std::string f(e);
    const std::string kind = f.substr(0, f.find(':'));
    fault_kind_ = kind == "grad" ? 1 : kind == "pull" ? 2 : kind == "param" ? 3 : kind == "drop" ? 4
                  : kind == "badpull" ? 5 : 0;
    // badpull: every one-sided pull (datapaths 0-2) this server serves to client
    // MPIT_PS_FAULT_CLIENT arrives with a corrupted first word (a broken (worker, server)
    // peer path for the pre-flight check; the two-sided datapath 3 stays intact)
    if (const char* c = std::getenv("MPIT_PS_FAULT_CLIENT")) fault_client_ = std::atoi(c);
    if (f.find(':') != std::string::npos) fault_at_ = std::max(1, std::atoi(f.c_str() + f.find(':') + 1));
    if (const char* r = std::getenv("MPIT_PS_FAULT_RANK"))
      if (std::atoi(r) != eng_.rank()) fault_kind_ = 0;
  }
  clock_.assign(clients_.size(), 0);
  tpush_.assign(clients_.size(), 0);
  if (device_) {
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    int lo = 0, hi = 0;
    hipp(hipDeviceGetStreamPriorityRange(&lo, &hi), "priority range");
    hipp(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "server stream");
    if (datapath_ == 2 || datapath_ == 3) {
      const size_t nc = clients_.size();
      if (datapath_ == 2) {
        // link streams. A server co-located with a worker shares its process with the
        // compute, priority, side, server and engine streams; one link stream per client
        // would put 7 more on the 4 hardware queues a process gets (GPU_MAX_HW_QUEUES), and
        // queue oversubscription is what collapsed the 8-rank rehearsal
        // (profiles/collapse_8rank_1gpu_r03.md): there at most 2, shared round-robin. A
        // dedicated server (no compute of its own) keeps one per client, so one client's
        // transfers never queue behind another's. MPIT_PS_LINK_STREAMS=k overrides. The
        // per-client events keep every client's inbox / update / outbox order whatever
        // stream it shares. (Datapath 3 moves its data on the PS link's one stream.)
        const bool colocated = client_index(eng_.rank()) >= 0;
        size_t nl = colocated ? std::min<size_t>(nc, 2) : nc;
        if (const char* e = std::getenv("MPIT_PS_LINK_STREAMS"))
          if (std::atoi(e) > 0) nl = std::min(nc, size_t(std::atoi(e)));
        cstream_.resize(std::max<size_t>(nl, 1));
        for (auto& cs : cstream_) hipp(hipStreamCreateWithPriority(&cs, hipStreamNonBlocking, hi), "link stream");
      }
      ev_in_.resize(nc);
      ev_up_.resize(nc);
      ev_out_.resize(nc);
      for (size_t i = 0; i < nc; ++i) {
        hipp(hipEventCreateWithFlags(&ev_in_[i], hipEventDisableTiming), "event");
        hipp(hipEventCreateWithFlags(&ev_up_[i], hipEventDisableTiming), "event");
        hipp(hipEventCreateWithFlags(&ev_out_[i], hipEventDisableTiming), "event");
      }
      if (nc && len_ > 0) hipp(hipMalloc(reinterpret_cast<void**>(&stage_), nc * size_t(len_) * 8), "hipMalloc(stage)");
    }
  }
}

PSServer::~PSServer() {
  {
    std::lock_guard<std::mutex> g(g_local_mu);
    auto it = g_local_servers.find({ps_id_, eng_.rank()});
    if (it != g_local_servers.end() && it->second == this) g_local_servers.erase(it);
  }
  for (int t = 1; t <= 8; ++t) eng_.register_am(ps_am_id(ps_id_, t), [](const Msg&) {});
  if (fg_) {
    {
      std::lock_guard<std::mutex> g(fg_->mu);  // waits for a flush in progress
      fg_->s = nullptr;
    }
    eng_.remove_hook(hook_);
  }
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


PSServer* PSServer::local(int ps_id, int rank) {
  std::lock_guard<std::mutex> g(g_local_mu);
  auto it = g_local_servers.find({ps_id, rank});
  return it == g_local_servers.end() ? nullptr : it->second;
}

hipEvent_t PSClient::pop_gate() {
  std::lock_guard<std::mutex> g(dep_mu_);
  if (gates_.empty()) throw std::logic_error("mpit: a kPsGpuGate message without its gate event");
  hipEvent_t e = gates_.front();
  gates_.pop_front();
  return e;
}


// the co-located server's message, sent now: its stream waits on the gate event instead of
// this client's progress thread polling it (the push of the step's last shard is then queued
// while the backward still runs, and the replies come back without waiting for the GPU)
void PSClient::send_local(hipStream_t s, int k, int tag, int64_t flags) {
  hipp(hipSetDevice(eng_.device()), "hipSetDevice");
  hipEvent_t e = eng_.get_event();
  Engine::record_event(e, s);
  {
    std::lock_guard<std::mutex> g(dep_mu_);
    gates_.push_back(e);
  }
  send_entry(k, tag, flags | kPsGpuGate);
}

PSClient* PSClient::local(int ps_id, int rank) {
  std::lock_guard<std::mutex> g(g_local_mu);
  auto it = g_local_clients.find({ps_id, rank});
  return it == g_local_clients.end() ? nullptr : it->second;
}

void PSClient::add_gpu_dep(hipEvent_t e) {
  std::lock_guard<std::mutex> g(dep_mu_);
  deps_.push_back(e);
}

void PSClient::take_deps(hipStream_t s) {
  std::vector<hipEvent_t> d;
  {
    std::lock_guard<std::mutex> g(dep_mu_);
    d.swap(deps_);
  }
  if (d.empty()) return;
  hipp(hipSetDevice(eng_.device()), "hipSetDevice");
  for (auto e : d) {
    hipp(hipStreamWaitEvent(s, e, 0), "wait co-located update");
    eng_.put_event(e);  // (the wait is queued: re-recording the event later does not affect it)
  }
}

PSClient* PSServer::early_client(int c) const {
  if (!device_ || c != eng_.rank() || !local_events()) return nullptr;
  return PSClient::local(ps_id_, c);
}

void PSServer::finish_for(int c, std::function<void()> replies) {
  if (PSClient* l = early_client(c)) {
    hipEvent_t e = eng_.get_event();
    Engine::record_event(e, stream_);
    l->add_gpu_dep(e);  // (before the replies: the client's wait sees it once they are in)
    replies();
    return;
  }
  finish(std::move(replies));
}

void PSServer::finish_on(hipStream_t s, std::function<void()> then) {
  hipEvent_t ev = eng_.get_event();
  Engine::record_event(ev, s);
  eng_.track_copy(ev, std::move(then));
}

void PSServer::start() {
  if (datapath_ == 3 && !link_) throw std::invalid_argument("mpit: PS datapath 3 needs its link (set_link)");
  if (batch_ && device_ && (rule_.kind == 0 || rule_.kind == 1)) {
    fg_ = std::make_shared<FlushGate>();
    fg_->s = this;
    auto fg = fg_;
    hook_ = eng_.add_hook([fg]() {
      std::lock_guard<std::mutex> g(fg->mu);
      return fg->s ? fg->s->flush_grads() : false;
    });
  }
  for (int t : {kTagInit, kTagGrad, kTagParam, kTagHeader, kTagStop})
    eng_.register_am(ps_am_id(ps_id_, t), [this](const Msg& m) { on_msg(m); });
  if (device_ && stream_) {
    std::lock_guard<std::mutex> g(g_local_mu);
    g_local_servers[{ps_id_, eng_.rank()}] = this;
  }
}

bool PSServer::batchable(int c) const {
  return fg_ && datapath_ != 1 && !pipelined(client_index(c), c) && !messaged(client_index(c), c);
}

void PSServer::queue_grad(int c, bool pull, Sub sb) {
  if (maybe_fault(1)) return;
  for (const auto& q : pend_)
    if (q.sb.o < sb.o + sb.n && sb.o < q.sb.o + q.sb.n) {  // same elements: keep the order
      flush_grads();
      break;
    }
  if (pend_.size() >= 16) flush_grads();
  const int ci = client_index(c);
  bool defer_pull = false;
  if (ci >= 0) {
    if (sb.o + sb.n == len_) ++clock_[size_t(ci)];
    if (pull && staleness_ >= 0) {
      int64_t mn = clock_[0];
      for (auto x : clock_) mn = std::min(mn, x);
      defer_pull = clock_[size_t(ci)] - mn > staleness_;
    }
  }
  pend_.push_back({c, pull, defer_pull, sb});
}

bool PSServer::flush_grads() {
  if (pend_.empty()) return false;
  TraceRange tr("ps_server_update_batch");
  std::vector<PendingGrad> batch;
  batch.swap(pend_);
  hipp(hipSetDevice(eng_.device()), "hipSetDevice");
  const int64_t es = grad_bf16_ ? 2 : 4;
  // two launches at most: the pieces that also write the pulled parameters (fused out
  // operand), and the ones that do not
  for (int wo = 0; wo < 2; ++wo) {
    std::vector<int64_t> ns;
    std::vector<std::vector<uintptr_t>> ptrs;
    for (const auto& q : batch) {
      const bool out = q.pull && !q.defer;
      if (out != (wo == 1)) continue;
      const int m = member_of(q.c);
      const void* g = reinterpret_cast<const uint8_t*>(tx_.remote_ptr(m)) + (off_ + q.sb.o) * es;
      void* o = out ? reinterpret_cast<uint8_t*>(rx_.remote_ptr(m)) + (off_ + q.sb.o) * 4 : nullptr;
      ns.push_back(q.sb.n);
      ptrs.push_back(rule_ptrs(g, o, q.sb));
    }
    if (ns.empty()) continue;
    const uint32_t bf = grad_bf16_ ? 2u : 0u;
    const int v = wo ? kOut : 0;
    ServerRule r = rule_;
    r.lr = lr_.load(std::memory_order_relaxed);
    if (r.kind == 0) ew_update_multi(kApply, v, eng_.device(), stream_, ns, ptrs, bf, {r.a});
    else ew_update_multi(kRMSProp, v | kAdd, eng_.device(), stream_, ns, ptrs, bf, {r.decay, r.lr, r.mom, r.eps});
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (const auto& q : batch) {
      if (q.sb.o + q.sb.n == len_) version_.fetch_add(1);
      ++stats_.grads;
      if (q.pull && !q.defer) ++stats_.pulls;
      if (q.defer) {
        deferred_.push_back({q.c, q.sb});
        ++stats_.deferred;
      }
    }
    ++stats_.batches;
    if (batch.size() >= 2) ++stats_.multi;
  }
  std::vector<PendingGrad> remote;
  PSClient* lc = nullptr;
  for (const auto& q : batch) {
    if (PSClient* l = early_client(q.c)) lc = l;
    else remote.push_back(q);
  }
  if (lc) {  // the co-located client: its GPU waits on this event, its host need not
    hipEvent_t e = eng_.get_event();
    Engine::record_event(e, stream_);
    lc->add_gpu_dep(e);
    for (const auto& q : batch)
      if (early_client(q.c)) {
        reply(q.c, kTagGradTail);
        if (q.pull && !q.defer) reply(q.c, kTagSendParam);
      }
  }
  if (!remote.empty())
    finish([this, remote] {
      for (const auto& q : remote) {
        reply(q.c, kTagGradTail);
        if (q.pull && !q.defer) reply(q.c, kTagSendParam);
      }
    });
  release_deferred();
  return true;
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

Sub PSServer::sub_of(const Msg& m) const {
  if (m.aux2 <= 0) return Sub{0, len_};
  const Sub sb{m.aux1 - off_, m.aux2};
  if (sb.o < 0 || sb.o + sb.n > len_)
    throw std::out_of_range("mpit: PS message names elements [" + std::to_string(m.aux1) + ", " +
                            std::to_string(m.aux1 + m.aux2) + ") outside this server's shard");
  return sb;
}

bool PSServer::maybe_fault(int kind) {
  // drop (4): the Nth and every later gradient push is silently ignored (a stuck server)
  if (fault_kind_ == 4 && kind == 1) return fault_seen_.fetch_add(1) + 1 >= fault_at_;
  if (fault_kind_ == kind && fault_seen_.fetch_add(1) + 1 == fault_at_)
    throw std::runtime_error("PS server " + std::to_string(ps_id_) + " on rank " + std::to_string(eng_.rank()) +
                             ": injected fault (MPIT_PS_FAULT)");
  return false;
}

void PSServer::on_msg(const Msg& m) {
  const int tag = (m.tag - 4096) % 16;
  if ((tag == kTagGrad || tag == kTagHeader || tag == kTagParam) && (m.aux0 & kPsGpuGate)) {
    // sent before the co-located client's GPU work behind it finished: everything this
    // message makes stream_ do waits for that work (queued now, so a backlogged message
    // served later is ordered too)
    PSClient* l = PSClient::local(ps_id_, m.src);
    if (!l || !device_) throw std::logic_error("mpit: kPsGpuGate from a client that is not the co-located one");
    hipEvent_t e = l->pop_gate();
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    hipp(hipStreamWaitEvent(stream_, e, 0), "server waits client gate");
    eng_.put_event(e);
  }
  // asyncsgd/pserver.lua:152-158: the shard is initialised from the first client's
  // parameter push before any gradient or pull is served
  if (init_rank_ >= 0 && (tag == kTagGrad || tag == kTagHeader)) {
    backlog_.push_back(m);
    return;
  }
  const bool qgrad = tag == kTagGrad && batchable(m.src);
  if (!qgrad) flush_grads();  // every other message sees the queued updates applied first
  switch (tag) {
    case kTagInit:
      // a client's shard entry must lie inside this server's shard
      if (m.aux0 < off_ || m.aux0 + m.aux1 > off_ + len_)
        std::fprintf(stderr, "[mpit ps %d] client %d shard (%lld,%lld) outside server shard (%lld,%lld)\n", ps_id_,
                     m.src, (long long)m.aux0, (long long)m.aux1, (long long)off_, (long long)len_);
      break;
    case kTagParam: {
      const Sub sb = sub_of(m);
      const bool init_piece = init_rank_ >= 0 && m.src == init_rank_;
      auto init_done = [this, sb] {
        if ((init_left_ -= sb.n) <= 0) {
          init_rank_ = -1;
          std::vector<Msg> later;
          later.swap(backlog_);
          for (auto& x : later) on_msg(x);
        }
      };
      if (init_piece && messaged(client_index(m.src), m.src)) {
        // datapath 3: the shard holds the initial parameters only once their transfer's turn
        // came (host: once the message landed; device: once the copy is queued on stream_)
        TraceRange tr("ps_server_param");
        maybe_fault(3);
        param_msg(m.src, client_index(m.src), (m.aux0 & kPsFromRx) != 0, sb, init_done);
        break;
      }
      do_param(m.src, (m.aux0 & kPsFromRx) != 0, sb);
      if (init_piece) init_done();
      break;
    }
    case kTagGrad:
      if (qgrad) queue_grad(m.src, (m.aux0 & kPsWithPull) != 0, sub_of(m));
      else do_grad(m.src, (m.aux0 & kPsWithPull) != 0, sub_of(m));
      break;
    case kTagHeader: {
      const Sub sb = sub_of(m);
      const int ci = client_index(m.src);
      if (staleness_ >= 0 && ci >= 0) {
        int64_t mn = clock_[0];
        for (auto c : clock_) mn = std::min(mn, c);
        if (clock_[size_t(ci)] - mn > staleness_) {
          std::lock_guard<std::mutex> g(mu_);
          deferred_.push_back({m.src, sb});
          ++stats_.deferred;
          break;
        }
      }
      do_pull(m.src, sb);
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
  finish_on(stream_, std::move(then));
}

void PSServer::reply(int c, int tag) { eng_.send_am(c, ps_am_id(ps_id_, tag), nullptr, 0); }

std::vector<uintptr_t> PSServer::rule_ptrs(const void* g, void* out, Sub sb) const {
  auto P = [](const void* x) { return reinterpret_cast<uintptr_t>(x); };
  auto F = [&](void* x) { return P(static_cast<uint8_t*>(x) + sb.o * 4); };  // fp32 state at the piece
  std::vector<uintptr_t> ptrs{F(p_), P(g)};
  static const int need[] = {0, 3, 2, 2, 1, 2};
  for (size_t k = 0; k < st_.size(); ++k)
    if (int(k) < need[rule_.kind]) ptrs.push_back(F(st_[k]));
  if (out) ptrs.push_back(P(out));
  return ptrs;
}

void PSServer::apply_rule(const void* g, void* out, Sub sb, int ci) {
  const int dev = device_ ? eng_.device() : -1;
  const uint32_t bf = grad_bf16_ ? 2u : 0u;
  const int v = out ? kOut : 0;
  const std::vector<uintptr_t> ptrs = rule_ptrs(g, out, sb);
  ServerRule r = rule_;  // progress thread only; lr may be changed concurrently (set_lr)
  r.lr = lr_.load(std::memory_order_relaxed);
  // the rule's step counter advances once per client push, on its first piece; the later
  // pieces of that push (split shard entries) reuse the step their first piece took, even
  // when another client's push arrived in between
  int64_t tc = 0;
  if (r.kind >= 2) {
    if (sb.o == 0) {
      tc = t_.fetch_add(1) + 1;
      if (ci >= 0) tpush_[size_t(ci)] = tc;
    } else {
      tc = ci >= 0 && tpush_[size_t(ci)] > 0 ? tpush_[size_t(ci)] : t_.load();
    }
  }
  switch (r.kind) {
    case 0:
      ew_update(kApply, v, dev, stream_, sb.n, ptrs, bf, {r.a});
      break;
    case 1:
      ew_update(kRMSProp, v | kAdd, dev, stream_, sb.n, ptrs, bf, {r.decay, r.lr, r.mom, r.eps});
      break;
    case 2: {  // BiCNN/pserver.lua:147-154: bias correction on floor(t/stepDiv)+1
      const double k = double(tc / std::max<int64_t>(1, r.step_div) + 1);
      const double lr_t = r.lr * std::sqrt(1.0 - std::pow(double(r.b2), k)) / (1.0 - std::pow(double(r.b1), k));
      ew_update(kAdam, v, dev, stream_, sb.n, ptrs, bf, {r.b1, r.b2, r.eps, float(lr_t)});
      break;
    }
    case 3: {  // BiCNN/pserver.lua:163-170
      const double lr_t = r.lr / (1.0 - std::pow(double(r.b1), double(tc)));
      ew_update(kAdamax, v, dev, stream_, sb.n, ptrs, bf, {r.b1, r.b2, r.eps, float(lr_t)});
      break;
    }
    case 4: {  // BiCNN/pserver.lua:177-182 (clr on the count before this push)
      const float clr = float(r.lr / (1.0 + double(tc - 1) * r.lrd));
      ew_update(kAdagrad, v, dev, stream_, sb.n, ptrs, bf, {r.eps, clr});
      break;
    }
    case 5:  // BiCNN/pserver.lua:189-193
      ew_update(kAdadelta, v, dev, stream_, sb.n, ptrs, bf, {r.rho, r.eps, r.lr});
      break;
  }
  if (sb.o + sb.n == len_) version_.fetch_add(1);
}

void PSServer::do_param(int c, bool from_rx, Sub sb) {
  TraceRange tr("ps_server_param");
  maybe_fault(3);
  if (messaged(client_index(c), c)) {
    param_msg(c, client_index(c), from_rx, sb);
    return;
  }
  const int m = member_of(c);
  const Window& w = from_rx ? rx_ : tx_;  // rx is always fp32
  const bool bf = grad_bf16_ && !from_rx;
  const int64_t es = bf ? 2 : 4;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(w.remote_ptr(m)) + (off_ + sb.o) * es;
  if (!device_ && w.remote_device(m)) throw std::runtime_error("mpit: host server cannot read a device window");
  if (device_) hipp(hipSetDevice(eng_.device()), "hipSetDevice");
  // p (fp32) = pushed shard (fp32 | bf16): one copy / cast kernel, or a host loop
  ew_update(kCopy, 0, device_ ? eng_.device() : -1, stream_, sb.n,
            {reinterpret_cast<uintptr_t>(static_cast<uint8_t*>(p_) + sb.o * 4), reinterpret_cast<uintptr_t>(src)},
            bf ? 2u : 0u, {1.f});
  {
    std::lock_guard<std::mutex> g(mu_);
    ++stats_.param_pushes;
  }
  finish_for(c, [this, c] { reply(c, kTagParamTail); });
}

void PSServer::copy_out(int c, Sub sb) {
  const int m = member_of(c);
  uint8_t* dst = reinterpret_cast<uint8_t*>(rx_.remote_ptr(m)) + (off_ + sb.o) * 4;
  const uint8_t* src = static_cast<const uint8_t*>(p_) + sb.o * 4;
  if (device_) {
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    if (datapath_ != 1)
      ew_update(kCopy, 0, eng_.device(), stream_, sb.n, {reinterpret_cast<uintptr_t>(dst), reinterpret_cast<uintptr_t>(src)},
                0u, {1.f});
    else
      hipp(hipMemcpyAsync(dst, src, size_t(sb.n) * 4, hipMemcpyDefault, stream_), "param pull copy");
  } else {
    if (rx_.remote_device(m)) throw std::runtime_error("mpit: host server cannot write a device rx window");
    std::memcpy(dst, src, size_t(sb.n) * 4);
  }
}

void PSServer::do_pull(int c, Sub sb) {
  TraceRange tr("ps_server_pull");
  maybe_fault(2);
  const int ci = client_index(c);
  if (messaged(ci, c)) {
    pull_msg(c, ci, sb);
    return;
  }
  if (pipelined(ci, c)) {
    // snapshot the piece in update order on stream_, push it over the client's link
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    hipStream_t cs = link(ci);
    uint8_t* out = stage_ + size_t(ci) * size_t(len_) * 8 + size_t(len_) * 4 + size_t(sb.o) * 4;
    uint8_t* dst = reinterpret_cast<uint8_t*>(rx_.remote_ptr(member_of(c))) + (off_ + sb.o) * 4;
    const uint8_t* src = static_cast<const uint8_t*>(p_) + sb.o * 4;
    hipp(hipStreamWaitEvent(stream_, ev_out_[size_t(ci)], 0), "wait outbox free");
    ew_update(kCopy, 0, eng_.device(), stream_, sb.n, {reinterpret_cast<uintptr_t>(out), reinterpret_cast<uintptr_t>(src)},
              0u, {1.f});
    hipp(hipEventRecord(ev_up_[size_t(ci)], stream_), "record snapshot");
    hipp(hipStreamWaitEvent(cs, ev_up_[size_t(ci)], 0), "link waits snapshot");
    hipp(hipMemcpyAsync(dst, out, size_t(sb.n) * 4, hipMemcpyDefault, cs), "param push (link)");
    if (fault_kind_ == 5 && c == fault_client_) hipp(hipMemsetAsync(dst, 0x7f, 4, cs), "injected bad pull");
    hipp(hipEventRecord(ev_out_[size_t(ci)], cs), "record outbox sent");
    {
      std::lock_guard<std::mutex> g(mu_);
      ++stats_.pulls;
    }
    finish_on(cs, [this, c] { reply(c, kTagSendParam); });
    return;
  }
  copy_out(c, sb);
  if (fault_kind_ == 5 && c == fault_client_ && sb.n > 0) {
    uint8_t* dst = reinterpret_cast<uint8_t*>(rx_.remote_ptr(member_of(c))) + (off_ + sb.o) * 4;
    if (device_) hipp(hipMemsetAsync(dst, 0x7f, 4, stream_), "injected bad pull");
    else std::memset(dst, 0x7f, 4);
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    ++stats_.pulls;
  }
  finish_for(c, [this, c] { reply(c, kTagSendParam); });
}

void PSServer::do_grad(int c, bool pull, Sub sb) {
  TraceRange tr(pull ? "ps_server_update+pull" : "ps_server_update");
  if (maybe_fault(1)) return;
  const int m = member_of(c);
  const int64_t es = grad_bf16_ ? 2 : 4;
  const void* g = reinterpret_cast<const uint8_t*>(tx_.remote_ptr(m)) + (off_ + sb.o) * es;
  const int ci = client_index(c);
  bool defer_pull = false;
  if (ci >= 0) {
    // one push per client per step: counted on the piece that ends the shard
    if (sb.o + sb.n == len_) ++clock_[size_t(ci)];
    if (pull && staleness_ >= 0) {
      int64_t mn = clock_[0];
      for (auto x : clock_) mn = std::min(mn, x);
      defer_pull = clock_[size_t(ci)] - mn > staleness_;
    }
  }
  if (messaged(ci, c)) {
    grad_msg(c, ci, pull, defer_pull, sb);
    return;
  }
  if (!device_ && tx_.remote_device(m)) throw std::runtime_error("mpit: host server cannot read a device tx window");
  if (pipelined(ci, c)) {
    // link stream: pull the gradient piece into this client's inbox; stream_: fused update
    // (+ snapshot into the outbox when a pull is due); link stream: push the snapshot
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    const size_t k = size_t(ci);
    hipStream_t cs = link(ci);
    uint8_t* in = stage_ + k * size_t(len_) * 8 + size_t(sb.o * es);
    uint8_t* out = stage_ + k * size_t(len_) * 8 + size_t(len_) * 4 + size_t(sb.o) * 4;
    const bool push_back = pull && !defer_pull;
    hipp(hipMemcpyAsync(in, g, size_t(sb.n * es), hipMemcpyDefault, cs), "grad pull (link)");
    hipp(hipEventRecord(ev_in_[k], cs), "record inbox full");
    hipp(hipStreamWaitEvent(stream_, ev_in_[k], 0), "update waits inbox");
    if (push_back) hipp(hipStreamWaitEvent(stream_, ev_out_[k], 0), "update waits outbox free");
    apply_rule(in, push_back ? out : nullptr, sb, ci);
    hipp(hipEventRecord(ev_up_[k], stream_), "record update");
    hipp(hipStreamWaitEvent(cs, ev_up_[k], 0), "link waits update");  // inbox reusable after this
    if (push_back) {
      uint8_t* dst = reinterpret_cast<uint8_t*>(rx_.remote_ptr(m)) + (off_ + sb.o) * 4;
      hipp(hipMemcpyAsync(dst, out, size_t(sb.n) * 4, hipMemcpyDefault, cs), "param push (link)");
      hipp(hipEventRecord(ev_out_[k], cs), "record outbox sent");
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      ++stats_.grads;
      if (push_back) ++stats_.pulls;
      if (defer_pull) {
        deferred_.push_back({c, sb});
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
    fused_out = reinterpret_cast<uint8_t*>(rx_.remote_ptr(m)) + (off_ + sb.o) * 4;
  if (device_) {
    hipp(hipSetDevice(eng_.device()), "hipSetDevice");
    if (datapath_ == 1) {
      void* ib = static_cast<uint8_t*>(inbox_) + sb.o * es;
      hipp(hipMemcpyAsync(ib, g, size_t(sb.n * es), hipMemcpyDefault, stream_), "grad inbox copy");
      g = ib;
    }
  }
  apply_rule(g, fused_out, sb, ci);
  if (pull && !defer_pull && !fused_out) copy_out(c, sb);
  {
    std::lock_guard<std::mutex> lk(mu_);
    ++stats_.grads;
    if (pull && !defer_pull) ++stats_.pulls;
    if (defer_pull) {
      deferred_.push_back({c, sb});
      ++stats_.deferred;
    }
  }
  finish_for(c, [this, c, pull, defer_pull] {
    reply(c, kTagGradTail);
    if (pull && !defer_pull) reply(c, kTagSendParam);
  });
  release_deferred();
}

// ---- datapath 3: the shard's data as two-sided messages with a remote client (link.h) -----
// Every transfer is put in the instance's global order first (PsLink::order); this server's
// side is queued when its turn comes. Device: the link stream carries the RCCL ops, the
// update / snapshot kernels stay on stream_ (one stream per shard: every update of the shard
// serialised), events order the two. Host (no GPU): per-transfer buffers, the link's FIFO runs
// the receive, the update as a queued call, then the send — in the same order.

void PSServer::grad_msg(int c, int ci, bool pull, bool defer_pull, Sub sb) {
  const int64_t es = grad_bf16_ ? 2 : 4;
  const bool push_back = pull && !defer_pull;
  {
    std::lock_guard<std::mutex> lk(mu_);
    ++stats_.grads;
    if (push_back) ++stats_.pulls;
    if (defer_pull) {
      deferred_.push_back({c, sb});
      ++stats_.deferred;
    }
  }
  const int64_t goff = (off_ + sb.o) * es, roff = (off_ + sb.o) * 4;
  if (device_) {
    const size_t k = size_t(ci);
    uint8_t* in = stage_ + k * size_t(len_) * 8 + size_t(sb.o * es);
    uint8_t* out = stage_ + k * size_t(len_) * 8 + size_t(len_) * 4 + size_t(sb.o) * 4;
    link_->order(c, false, 1, goff, sb.n * es, [this, c, ci, k, in, out, sb, es, push_back] {
      hipp(hipSetDevice(eng_.device()), "hipSetDevice");
      link_->recv(c, in, sb.n * es, ev_up_[k]);  // the inbox is free once the last update read it
      link_->record(ev_in_[k]);
      hipp(hipStreamWaitEvent(stream_, ev_in_[k], 0), "update waits inbox");
      if (push_back) hipp(hipStreamWaitEvent(stream_, ev_out_[k], 0), "update waits outbox free");
      apply_rule(in, push_back ? out : nullptr, sb, ci);
      hipp(hipEventRecord(ev_up_[k], stream_), "record update");
      if (!push_back) finish_on(stream_, [this, c] { reply(c, kTagGradTail); });
    });
    if (push_back)
      link_->order(c, true, 0, roff, sb.n * 4, [this, c, k, out, sb] {
        link_->send(c, out, sb.n * 4, ev_up_[k]);
        link_->record(ev_out_[k]);
        link_->then([this, c] {
          reply(c, kTagGradTail);
          reply(c, kTagSendParam);
        });
      });
  } else {
    auto in = std::make_shared<std::vector<uint8_t>>(size_t(sb.n * es));
    auto out = push_back ? std::make_shared<std::vector<uint8_t>>(size_t(sb.n) * 4) : nullptr;
    link_->order(c, false, 1, goff, sb.n * es, [this, c, ci, sb, es, in, out, push_back] {
      link_->recv(c, in->data(), sb.n * es);
      link_->call([this, c, ci, sb, in, out, push_back] {
        apply_rule(in->data(), out ? out->data() : nullptr, sb, ci);
        if (!push_back) reply(c, kTagGradTail);
      });
    });
    if (push_back)
      link_->order(c, true, 0, roff, sb.n * 4, [this, c, sb, out] {
        link_->send(c, out->data(), sb.n * 4);
        link_->call([this, c, out] {
          reply(c, kTagGradTail);
          reply(c, kTagSendParam);
        });
      });
  }
  // pulls released by this push are ordered after it: their snapshots see its update
  release_deferred();
}

void PSServer::pull_msg(int c, int ci, Sub sb) {
  {
    std::lock_guard<std::mutex> g(mu_);
    ++stats_.pulls;
  }
  const int64_t roff = (off_ + sb.o) * 4;
  if (device_) {
    const size_t k = size_t(ci);
    uint8_t* out = stage_ + k * size_t(len_) * 8 + size_t(len_) * 4 + size_t(sb.o) * 4;
    link_->order(c, true, 0, roff, sb.n * 4, [this, c, k, out, sb] {
      hipp(hipSetDevice(eng_.device()), "hipSetDevice");
      const uint8_t* src = static_cast<const uint8_t*>(p_) + sb.o * 4;
      // the snapshot in update order on stream_, sent on the link stream
      hipp(hipStreamWaitEvent(stream_, ev_out_[k], 0), "wait outbox free");
      ew_update(kCopy, 0, eng_.device(), stream_, sb.n, {reinterpret_cast<uintptr_t>(out), reinterpret_cast<uintptr_t>(src)},
                0u, {1.f});
      hipp(hipEventRecord(ev_up_[k], stream_), "record snapshot");
      link_->send(c, out, sb.n * 4, ev_up_[k]);
      link_->record(ev_out_[k]);
      link_->then([this, c] { reply(c, kTagSendParam); });
    });
    return;
  }
  auto out = std::make_shared<std::vector<uint8_t>>(size_t(sb.n) * 4);
  link_->order(c, true, 0, roff, sb.n * 4, [this, c, sb, out] {
    // host: the snapshot is taken when the FIFO reaches it, after every update queued before
    link_->call([this, sb, out] { std::memcpy(out->data(), static_cast<const uint8_t*>(p_) + sb.o * 4, size_t(sb.n) * 4); });
    link_->send(c, out->data(), sb.n * 4);
    link_->call([this, c, out] { reply(c, kTagSendParam); });
  });
}

void PSServer::param_msg(int c, int ci, bool from_rx, Sub sb, std::function<void()> after) {
  const bool bf = grad_bf16_ && !from_rx;
  const int64_t es = bf ? 2 : 4;
  {
    std::lock_guard<std::mutex> g(mu_);
    ++stats_.param_pushes;
  }
  const int64_t coff = (off_ + sb.o) * es;
  if (device_) {
    const size_t k = size_t(ci);
    uint8_t* in = stage_ + k * size_t(len_) * 8 + size_t(sb.o * es);
    link_->order(c, false, from_rx ? 0 : 1, coff, sb.n * es, [this, c, k, in, sb, es, bf, after] {
      hipp(hipSetDevice(eng_.device()), "hipSetDevice");
      link_->recv(c, in, sb.n * es, ev_up_[k]);
      link_->record(ev_in_[k]);
      hipp(hipStreamWaitEvent(stream_, ev_in_[k], 0), "copy waits inbox");
      ew_update(kCopy, 0, eng_.device(), stream_, sb.n,
                {reinterpret_cast<uintptr_t>(static_cast<uint8_t*>(p_) + sb.o * 4), reinterpret_cast<uintptr_t>(in)},
                bf ? 2u : 0u, {1.f});
      hipp(hipEventRecord(ev_up_[k], stream_), "record copy");
      finish([this, c] { reply(c, kTagParamTail); });
      // an initialising push: the backlog (local fused updates included) queues behind the copy
      if (after) after();
    });
    return;
  }
  auto in = std::make_shared<std::vector<uint8_t>>(size_t(sb.n * es));
  link_->order(c, false, from_rx ? 0 : 1, coff, sb.n * es, [this, c, sb, es, in, bf, after] {
    link_->recv(c, in->data(), sb.n * es);
    link_->call([this, c, sb, in, bf, after] {
      ew_update(kCopy, 0, -1, nullptr, sb.n,
                {reinterpret_cast<uintptr_t>(static_cast<uint8_t*>(p_) + sb.o * 4), reinterpret_cast<uintptr_t>(in->data())},
                bf ? 2u : 0u, {1.f});
      reply(c, kTagParamTail);
      if (after) after();
    });
  });
}

void PSServer::release_deferred() {
  if (staleness_ < 0) return;
  std::deque<std::pair<int, Sub>> ready;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (deferred_.empty()) return;
    int64_t mn = clock_.empty() ? 0 : clock_[0];
    for (auto x : clock_) mn = std::min(mn, x);
    std::deque<std::pair<int, Sub>> keep;
    for (auto& d : deferred_) {
      const int ci = client_index(d.first);
      if (ci < 0 || clock_[size_t(ci)] - mn <= staleness_) ready.push_back(d);
      else keep.push_back(d);
    }
    deferred_.swap(keep);
  }
  for (auto& d : ready) do_pull(d.first, d.second);
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

bool PSClient::gpu_gate(int k) const {
  if (eng_.device() < 0 || link_ || servers_[size_t(k)] != eng_.rank() || !local_events() || !local_gate() ||
      PSServer::local(ps_id_, eng_.rank()) == nullptr)
    return false;
  // an entry still waiting in the gate queue may be for this server: keep the call order
  std::lock_guard<std::mutex> l(gq_->mu);
  return gq_->q.empty();
}

PSClient::PSClient(Engine& eng, int ps_id, std::vector<int> servers, std::vector<int64_t> offs,
                   std::vector<int64_t> lens)
    : eng_(eng), ps_id_(ps_id), servers_(std::move(servers)), offs_(std::move(offs)), lens_(std::move(lens)) {
  if (servers_.size() != offs_.size() || servers_.size() != lens_.size())
    throw std::invalid_argument("mpit: PSClient shard table mismatch");
  auto gq = std::make_shared<GateQueue>();
  gq_ = gq;
  Engine* e = &eng_;
  hook_ = eng_.add_hook([gq, e]() {
    bool did = false;
    for (;;) {
      GateQueue::Gate g;
      {
        std::lock_guard<std::mutex> l(gq->mu);
        if (gq->q.empty()) break;
        g = gq->q.front();
        if (g.ev) {
          hipSetDevice(e->device());
          const hipError_t st = hipEventQuery(g.ev);
          if (st == hipErrorNotReady) break;
          if (st != hipSuccess)
            throw std::runtime_error(std::string("PS client gate: GPU work before a push failed: ") +
                                     hipGetErrorString(st));
        }
        gq->q.pop_front();
      }
      if (g.ev) {
        e->put_event(g.ev);
        e->gpu_pending_add(-1);
      }
      g.send();
      did = true;
    }
    return did;
  });
}

PSClient::~PSClient() {
  {
    std::lock_guard<std::mutex> g(g_local_mu);
    auto it = g_local_clients.find({ps_id_, eng_.rank()});
    if (it != g_local_clients.end() && it->second == this) g_local_clients.erase(it);
  }
  {
    std::lock_guard<std::mutex> g(dep_mu_);
    for (auto e : deps_) eng_.put_event(e);
    deps_.clear();
    for (auto e : gates_) eng_.put_event(e);
    gates_.clear();
  }
  if (hook_ >= 0) eng_.remove_hook(hook_);
  if (link_) link_->set_client(nullptr);
  // gates never retired (the client went away with pushes queued): release their events
  // and their pending count, or deep parking stays disabled for the rest of the process
  std::deque<GateQueue::Gate> left;
  {
    std::lock_guard<std::mutex> l(gq_->mu);
    left.swap(gq_->q);
  }
  for (auto& g : left)
    if (g.ev) {
      hipEventSynchronize(g.ev);
      eng_.put_event(g.ev);
      eng_.gpu_pending_add(-1);
    }
}

void PSClient::start() {
  if (eng_.device() >= 0) {
    std::lock_guard<std::mutex> g(g_local_mu);
    g_local_clients[{ps_id_, eng_.rank()}] = this;
  }
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
    g.ev = eng_.get_event();
    Engine::record_event(g.ev, s);
  }
  // count the pending GPU event BEFORE the gate becomes visible to the progress hook: the
  // hook may pop it (and decrement) right after the push, and an under-count while another
  // gate is outstanding would let the progress thread park with an event still to poll
  if (g.ev) eng_.gpu_pending_add(1);
  {
    std::lock_guard<std::mutex> l(gq_->mu);
    gq_->q.push_back(g);
  }
  if (!g.ev) eng_.kick();
}

void PSClient::set_link(PsLink* l, uintptr_t rx, uintptr_t tx, int tx_es) {
  link_ = l;
  rx_ = reinterpret_cast<uint8_t*>(rx);
  tx_ = reinterpret_cast<uint8_t*>(tx);
  tx_es_ = tx_es;
  if (!l) return;
  // this client's side of a transfer, queued at its turn in the instance's order (link.h)
  l->set_client([this](int server, bool to_client, int window, int64_t coff, int64_t bytes) {
    uint8_t* base = window == 0 ? rx_ : tx_;
    if (to_client) {
      link_->recv(server, base + coff, bytes);
      link_->then([this] { local_done(); });  // the shard has landed in rx
    } else {
      link_->send(server, base + coff, bytes);
    }
  });
}

int PSClient::link_recvs(int k, int tag, int64_t flags) const {
  if (!link_ || (servers_[size_t(k)] == eng_.rank() && !PsLink::self_mode())) return 0;
  return (tag == kTagHeader || (tag == kTagGrad && (flags & kPsWithPull))) ? 1 : 0;
}

void PSClient::local_done() {
  pending_.fetch_sub(1, std::memory_order_seq_cst);
  reply_seq_.fetch_add(1, std::memory_order_seq_cst);
  futex_wake_all(&reply_seq_, false);
}

void PSClient::send_entry(int k, int tag, int64_t flags) {
  const int srv = servers_[size_t(k)];
  const bool whole = std::count(servers_.begin(), servers_.end(), srv) == 1;
  eng_.send_am(srv, ps_am_id(ps_id_, tag), nullptr, 0, flags, whole ? 0 : offs_[size_t(k)], whole ? 0 : lens_[size_t(k)]);
  // datapath 3: the server puts the entry's data in the instance's order (PsLink::order); the
  // pre-sequencer layout (MPIT_LINK_LEGACY, host tests only) queued it here, in call order
  if (!link_ || srv == eng_.rank() || !link_->legacy()) return;
  const int64_t o = offs_[size_t(k)], n = lens_[size_t(k)];
  if (tag == kTagGrad) {
    link_->send(srv, tx_ + o * tx_es_, n * tx_es_);
  } else if (tag == kTagParam) {
    if (flags & kPsFromRx) link_->send(srv, rx_ + o * 4, n * 4);
    else link_->send(srv, tx_ + o * tx_es_, n * tx_es_);
  }
  if (link_recvs(k, tag, flags)) {
    link_->recv(srv, rx_ + o * 4, n * 4);
    link_->then([this] { local_done(); });
  }
}

// Entries of the co-located device server go out at once with a gate event (send_local);
// the others wait in the gate queue for the GPU work queued so far on s. (Per server the
// call order is kept either way: a server's entries all take the same route.)
void PSClient::send_grad(hipStream_t s, bool with_pull) {
  const int64_t n = int64_t(servers_.size());
  int64_t extra = 0;
  for (int k = 0; k < int(n); ++k) extra += link_recvs(k, kTagGrad, with_pull ? kPsWithPull : 0);
  pending_.fetch_add((with_pull ? 2 * n : n) + extra);
  const int64_t fl = with_pull ? kPsWithPull : 0;
  std::vector<int> gated;
  for (int k = 0; k < int(n); ++k) {
    if (gpu_gate(k)) send_local(s, k, kTagGrad, fl);
    else gated.push_back(k);
  }
  if (!gated.empty())
    gate(s, [this, gated, fl] {
      for (int k : gated) send_entry(k, kTagGrad, fl);
    });
}

void PSClient::send_grad_to(hipStream_t s, int k, bool with_pull) {
  if (k < 0 || k >= int(servers_.size())) throw std::out_of_range("PSClient::send_grad_to: bad shard");
  pending_.fetch_add((with_pull ? 2 : 1) + link_recvs(k, kTagGrad, with_pull ? kPsWithPull : 0));
  if (gpu_gate(k)) {
    send_local(s, k, kTagGrad, with_pull ? kPsWithPull : 0);
    return;
  }
  gate(s, [this, k, with_pull] { send_entry(k, kTagGrad, with_pull ? kPsWithPull : 0); });
}

void PSClient::recv_param(hipStream_t s) {
  const int n = int(servers_.size());
  int64_t extra = 0;
  for (int k = 0; k < n; ++k) extra += link_recvs(k, kTagHeader, 0);
  pending_.fetch_add(n + extra);
  // ordered behind any gated push of this client
  std::vector<int> gated;
  for (int k = 0; k < n; ++k) {
    if (gpu_gate(k)) send_local(s, k, kTagHeader, 0);
    else gated.push_back(k);
  }
  if (!gated.empty())
    gate(s, [this, gated] {
      for (int k : gated) send_entry(k, kTagHeader, 0);
    });
}

void PSClient::send_param(hipStream_t s, bool from_rx) {
  const int n = int(servers_.size());
  pending_.fetch_add(n);
  const int64_t fl = from_rx ? kPsFromRx : 0;
  std::vector<int> gated;
  for (int k = 0; k < n; ++k) {
    if (gpu_gate(k)) send_local(s, k, kTagParam, fl);
    else gated.push_back(k);
  }
  if (!gated.empty())
    gate(s, [this, gated, fl] {
      for (int k : gated) send_entry(k, kTagParam, fl);
    });
}

void PSClient::stop() {
  wait();
  std::vector<int> done;
  for (int srv : servers_) {  // one stop per server, however many entries it has
    if (std::find(done.begin(), done.end(), srv) != done.end()) continue;
    done.push_back(srv);
    eng_.send_am(srv, ps_am_id(ps_id_, kTagStop), nullptr, 0);
  }
}

void PSClient::on_reply(const Msg&) {
  replies_.fetch_add(1);
  pending_.fetch_sub(1, std::memory_order_seq_cst);
  reply_seq_.fetch_add(1, std::memory_order_seq_cst);
  futex_wake_all(&reply_seq_, false);
}

// The worker waits here every step while the GPU finishes its backward (tens of ms).
// MPIT_WAIT_SPIN_US > 0 polls (pause) for up to that long before the futex sleep, keeping
// the core awake for the step start that follows (device clients only). Measured within
// noise of sleeping at once (profiles/step_start_host_r02.md): default 0.
// MPIT_PS_TIMEOUT_S (default 0 = never, opt-in on every datapath): a reply missing that long
// means a server is gone or stuck — raise with what is missing instead of hanging the job (a
// server that fails raises the job-wide abort itself, Engine::fatal; a dead server process is
// caught by the peer check). Off by default: an SSP-deferred pull may wait on a slow
// straggler (validation, checkpointing) for as long as that straggler takes, as the
// reference's blocking MPI calls do. bench.py opts in (300 s) for its own runs.
void PSClient::wait() {
  static const int64_t spin_us = [] {
    const char* e = std::getenv("MPIT_WAIT_SPIN_US");
    return e ? std::max<int64_t>(0, std::atoll(e)) : int64_t(0);
  }();
  static const double timeout_s = [] {
    const char* e = std::getenv("MPIT_PS_TIMEOUT_S");
    return e ? std::max(0.0, std::atof(e)) : 0.0;
  }();
  const auto t0 = std::chrono::steady_clock::now();
  if (spin_us > 0 && eng_.device() >= 0) {  // GPU workers only (CPU ranks share few cores)
    for (uint32_t i = 0;; ++i) {
      if (pending_.load(std::memory_order_acquire) <= 0) return;
      _mm_pause();
      if ((i & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us)) break;
    }
  }
  for (;;) {
    const uint32_t seq = reply_seq_.load(std::memory_order_seq_cst);
    const int64_t v = pending_.load(std::memory_order_seq_cst);
    if (v <= 0) return;
    int64_t slice_us = 1000000;
    if (timeout_s > 0) {
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el >= timeout_s) {
        std::string srv;
        for (size_t k = 0; k < servers_.size(); ++k) srv += (k ? "," : "") + std::to_string(servers_[k]);
        throw std::runtime_error("mpit: PS client " + std::to_string(eng_.rank()) + " waited " +
                                 std::to_string(int(timeout_s)) + " s for " + std::to_string(v) +
                                 " server replies (servers " + srv + ", ps " + std::to_string(ps_id_) +
                                 "); a server is gone or stuck (MPIT_PS_TIMEOUT_S)");
      }
      slice_us = std::min<int64_t>(slice_us, int64_t((timeout_s - el) * 1e6) + 1);
    }
    futex_wait(&reply_seq_, seq, slice_us, false);
  }
}

}  // namespace mpit
