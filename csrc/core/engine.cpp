#include "engine.h"

#include <linux/futex.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <xmmintrin.h>

#include <climits>
#include <ctime>

#include <algorithm>
#include <cerrno>
#include <csignal>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace mpit {

namespace {
void hipc(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("mpit engine HIP error in ") + what + ": " + hipGetErrorString(e));
}

double env_seconds(const char* name, double dflt) {
  const char* e = std::getenv(name);
  return e ? std::max(0.0, std::atof(e)) : dflt;
}
}  // namespace

void futex_wake_all(void* addr, bool shared) {
  ::syscall(SYS_futex, addr, shared ? FUTEX_WAKE : FUTEX_WAKE_PRIVATE, INT_MAX, nullptr, nullptr, 0);
}

void futex_wait(void* addr, uint32_t expect, int64_t timeout_us, bool shared) {
  timespec ts{};
  timespec* tp = nullptr;
  if (timeout_us >= 0) {
    ts.tv_sec = time_t(timeout_us / 1000000);
    ts.tv_nsec = long(timeout_us % 1000000) * 1000L;
    tp = &ts;
  }
  ::syscall(SYS_futex, addr, shared ? FUTEX_WAIT : FUTEX_WAIT_PRIVATE, expect, tp, nullptr, 0);
}

double Engine::wait_timeout_s() {
  // 0 (default) = never: MPI's blocking calls have no deadline either, and a rank may
  // legitimately sit in Barrier / Wait for hours (a BiCNN rank outside the active set, a fast
  // goot worker at the final Barrier). Dead peers are caught by check_peers + the abort flag;
  // tests opt in to a deadline.
  static const double t = env_seconds("MPIT_WAIT_TIMEOUT_S", 0.0);
  return t;
}

Engine::Engine(const std::string& shm_name, int world, int rank, bool create, int device, int64_t bulk_bytes)
    : world_(world), rank_(rank), device_(device) {
  seg_ = std::make_unique<Segment>(shm_name, world, rank, create, bulk_bytes);
  sendq_.resize(world);
  ctrlq_.resize(world);
  streaming_.resize(world);
  send_seq_.assign(world, 0);
  auto& ri = seg_->hdr()->ranks[rank];
  ri.pid = int32_t(::getpid());
  ri.device = device;
  ::gethostname(ri.host, sizeof(ri.host) - 1);
  ri.attached.store(1, std::memory_order_release);
  seg_->hdr()->nattached.fetch_add(1, std::memory_order_acq_rel);
  if (device_ >= 0) {
    hipc(hipSetDevice(device_), "hipSetDevice");
    int lo = 0, hi = 0;
    hipc(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
    hipc(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "hipStreamCreateWithPriority");
  }
  thread_ = std::thread([this] { progress_loop(); });
}

Engine::~Engine() {
  try {
    shutdown();
  } catch (...) {
  }
}

void Engine::shutdown() {
  if (!running_.exchange(false)) return;
  // a clean exit: peers must not take this rank's disappearance for a crash
  seg_->hdr()->ranks[rank_].attached.store(2, std::memory_order_release);
  if (thread_.joinable()) thread_.join();
  if (device_ >= 0) {
    hipSetDevice(device_);
    {
      std::lock_guard<std::mutex> g(copy_mu_);
      for (auto& c : copies_) {
        hipEventSynchronize(c.ev);
        hipEventDestroy(c.ev);
      }
      copies_.clear();
    }
    {
      std::lock_guard<std::mutex> g(ev_mu_);
      for (auto e : ev_pool_) hipEventDestroy(e);
      ev_pool_.clear();
    }
    {
      std::lock_guard<std::mutex> g(ipc_mu_);
      for (auto& kv : ipc_cache_) hipIpcCloseMemHandle(kv.second.ptr);
      ipc_cache_.clear();
    }
    if (stream_) hipStreamDestroy(stream_);
    stream_ = nullptr;
  }
}

// --------------------------------------------------------------------------- utilities

std::shared_ptr<Req> Engine::get_req(int64_t id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = reqs_.find(id);
  if (it == reqs_.end()) throw std::invalid_argument("mpit: unknown or already freed request " + std::to_string(id));
  return it->second;
}

void Engine::finish_req(const std::shared_ptr<Req>& r, int state) {
  r->state.store(state, std::memory_order_seq_cst);
  futex_wake_all(&r->state, false);
}

bool Engine::match(const Msg& h, const Req& r) const {
  return h.ctx == r.ctx && (r.src == kAnySource || r.src == h.src) && (r.tag == kAnyTag || r.tag == h.tag);
}

bool Engine::push_msg_locked(int dst, const Msg& m) {
  Ring* ring = seg_->ring(rank_, dst);
  const uint64_t head = ring->head.load(std::memory_order_relaxed);
  const uint64_t tail = ring->tail.load(std::memory_order_acquire);
  if (head - tail >= uint64_t(kRingSlots)) return false;
  ring->slots[head % kRingSlots] = m;
  ring->head.store(head + 1, std::memory_order_seq_cst);
  msgs_sent_.fetch_add(1, std::memory_order_relaxed);
  this->ring(dst);
  return true;
}

int64_t Engine::bulk_write_locked(int dst, const uint8_t* p, int64_t n) {
  BulkHdr* b = seg_->bulk(rank_, dst);
  uint8_t* data = seg_->bulk_data(rank_, dst);
  const int64_t cap = seg_->bulk_bytes();
  const uint64_t w = b->wpos.load(std::memory_order_relaxed);
  const uint64_t r = b->rpos.load(std::memory_order_acquire);
  const int64_t free = cap - int64_t(w - r);
  const int64_t m = std::min(n, free);
  if (m <= 0) return 0;
  const int64_t off = int64_t(w % uint64_t(cap));
  const int64_t first = std::min(m, cap - off);
  std::memcpy(data + off, p, size_t(first));
  if (m > first) std::memcpy(data, p + first, size_t(m - first));
  b->wpos.store(w + uint64_t(m), std::memory_order_seq_cst);
  ring(dst);
  return m;
}

int64_t Engine::bulk_read(int src, uint8_t* p, int64_t n) {
  BulkHdr* b = seg_->bulk(src, rank_);
  const uint8_t* data = seg_->bulk_data(src, rank_);
  const int64_t cap = seg_->bulk_bytes();
  const uint64_t r = b->rpos.load(std::memory_order_relaxed);
  const uint64_t w = b->wpos.load(std::memory_order_acquire);
  const int64_t avail = int64_t(w - r);
  const int64_t m = std::min(n, avail);
  if (m <= 0) return 0;
  const int64_t off = int64_t(r % uint64_t(cap));
  const int64_t first = std::min(m, cap - off);
  std::memcpy(p, data + off, size_t(first));
  if (m > first) std::memcpy(p + first, data, size_t(m - first));
  b->rpos.store(r + uint64_t(m), std::memory_order_seq_cst);
  ring(src);  // the sender may be waiting for space
  return m;
}

void Engine::export_ptr(const void* p, hipIpcMemHandle_t* h, int64_t* offset, int64_t* alloc_bytes) {
  hipDeviceptr_t base = nullptr;
  size_t sz = 0;
  hipc(hipMemGetAddressRange(&base, &sz, const_cast<void*>(p)), "hipMemGetAddressRange");
  hipc(hipIpcGetMemHandle(h, base), "hipIpcGetMemHandle");
  *offset = int64_t(reinterpret_cast<const uint8_t*>(p) - reinterpret_cast<const uint8_t*>(base));
  if (alloc_bytes) *alloc_bytes = int64_t(sz);
}

void Engine::export_cached(const void* p, hipIpcMemHandle_t* h, int64_t* offset) {
  hipDeviceptr_t base = nullptr;
  size_t sz = 0;
  hipc(hipMemGetAddressRange(&base, &sz, const_cast<void*>(p)), "hipMemGetAddressRange");
  uint64_t id = 0;
  hipc(hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(p))),
       "hipPointerGetAttribute(BUFFER_ID)");
  *offset = int64_t(reinterpret_cast<const uint8_t*>(p) - reinterpret_cast<const uint8_t*>(base));
  std::lock_guard<std::mutex> g(export_mu_);
  auto it = export_cache_.find(id);
  if (it != export_cache_.end() && it->second.second == reinterpret_cast<uintptr_t>(base)) {
    *h = it->second.first;
    return;
  }
  hipc(hipIpcGetMemHandle(h, base), "hipIpcGetMemHandle");
  if (export_cache_.size() > 4096) export_cache_.clear();  // bounded; entries are cheap to redo
  export_cache_[id] = {*h, reinterpret_cast<uintptr_t>(base)};
}

void* Engine::open_ipc(int owner_rank, const hipIpcMemHandle_t& h, bool permanent) {
  std::string key(reinterpret_cast<const char*>(&h), sizeof(h));
  std::lock_guard<std::mutex> g(ipc_mu_);
  auto it = ipc_cache_.find({owner_rank, key});
  if (it != ipc_cache_.end()) {
    it->second.last_use = ++ipc_tick_;
    it->second.inflight += permanent ? kPinned : 1;
    return it->second.ptr;
  }
  if (ipc_cache_.size() >= kIpcCacheMax) {  // close the least recently used idle mapping
    auto victim = ipc_cache_.end();
    for (auto v = ipc_cache_.begin(); v != ipc_cache_.end(); ++v)
      if (v->second.inflight == 0 && (victim == ipc_cache_.end() || v->second.last_use < victim->second.last_use))
        victim = v;
    if (victim != ipc_cache_.end()) {
      hipIpcCloseMemHandle(victim->second.ptr);
      ipc_cache_.erase(victim);
    }
  }
  hipc(hipSetDevice(device_), "hipSetDevice");
  void* p = nullptr;
  hipc(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  IpcMapping mp;
  mp.ptr = p;
  mp.last_use = ++ipc_tick_;
  mp.inflight = permanent ? kPinned : 1;
  ipc_cache_[{owner_rank, key}] = mp;
  return p;
}

void Engine::release_ipc(int owner_rank, const std::string& key) {
  std::lock_guard<std::mutex> g(ipc_mu_);
  auto it = ipc_cache_.find({owner_rank, key});
  if (it != ipc_cache_.end() && it->second.inflight > 0) --it->second.inflight;
}

// --------------------------------------------------------------------------- p2p API

int64_t Engine::isend(const void* buf, int64_t nbytes, bool dev, int dst, int tag, int ctx, bool sync) {
  if (dst < 0 || dst >= world_) throw std::invalid_argument("mpit: invalid destination rank");
  if (dev && device_ < 0) throw std::invalid_argument("mpit: device buffer on a rank without a device");
  auto r = std::make_shared<Req>();
  r->id = next_id_.fetch_add(1);
  r->is_send = true;
  r->dst = dst;
  r->sbuf = static_cast<const uint8_t*>(buf);
  r->nbytes = nbytes;
  r->sdev = dev;
  r->sdevice = device_;
  r->sync = sync;
  r->tag = tag;
  r->ctx = ctx;
  r->st.source = rank_;
  r->st.tag = tag;
  r->st.count = nbytes;
  std::lock_guard<std::mutex> g(mu_);
  reqs_[r->id] = r;
  sendq_[dst].push_back(r);
  kick();
  return r->id;
}

int64_t Engine::irecv(void* buf, int64_t cap, bool dev, int src, int tag, int ctx) {
  if (src != kAnySource && (src < 0 || src >= world_)) throw std::invalid_argument("mpit: invalid source rank");
  if (dev && device_ < 0) throw std::invalid_argument("mpit: device buffer on a rank without a device");
  auto r = std::make_shared<Req>();
  r->id = next_id_.fetch_add(1);
  r->rbuf = static_cast<uint8_t*>(buf);
  r->cap = cap;
  r->rdev = dev;
  r->rdevice = device_;
  r->src = src;
  r->tag = tag;
  r->ctx = ctx;
  std::lock_guard<std::mutex> g(mu_);
  reqs_[r->id] = r;
  for (auto it = unexpected_.begin(); it != unexpected_.end(); ++it) {
    auto in = *it;
    if (!match(in->hdr, *r)) continue;
    unexpected_.erase(it);
    in->req = r;
    if (in->hdr.kind == MK_DEV) {
      start_dev_pull_locked(*in);
    } else if (in->complete) {
      deliver_locked(*in);
    }  // else: still streaming into in->data; delivered on completion
    return r->id;
  }
  posted_.push_back(r);
  kick();
  return r->id;
}

bool Engine::test(int64_t id, Status* st, bool keep) {
  auto r = get_req(id);
  const int s = r->state.load(std::memory_order_acquire);
  if (s == RS_PENDING) return false;
  if (s == RS_ERROR) {
    if (!keep) free_request(id);
    throw std::runtime_error("mpit: request failed: " + r->err);
  }
  if (st) *st = r->st;
  if (!keep) free_request(id);
  return true;
}

void Engine::wait(int64_t id, Status* st) {
  auto r = get_req(id);
  const double tmo = wait_timeout_s();
  const auto t0 = std::chrono::steady_clock::now();
  while (r->state.load(std::memory_order_seq_cst) == RS_PENDING) {
    int64_t left_us = -1;
    if (tmo > 0) {
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el >= tmo)
        throw std::runtime_error("mpit: Wait timed out after " + std::to_string(int(tmo)) + " s (" +
                                 (r->is_send ? "send to rank " + std::to_string(r->dst)
                                             : "receive from rank " + std::to_string(r->src)) +
                                 ", tag " + std::to_string(r->tag) + "; MPIT_WAIT_TIMEOUT_S)");
      left_us = int64_t((tmo - el) * 1e6) + 1;
    }
    // bounded slices: the abort flag of a failed peer is checked by the progress thread,
    // which _exits the process, so the slice only bounds the deadline check
    futex_wait(&r->state, RS_PENDING, left_us < 0 ? 1000000 : std::min<int64_t>(left_us, 1000000), false);
  }
  test(id, st, false);
}

void Engine::free_request(int64_t id) {
  std::lock_guard<std::mutex> g(mu_);
  reqs_.erase(id);
}

bool Engine::cancel(int64_t id) {
  auto r = get_req(id);
  std::lock_guard<std::mutex> g(mu_);
  if (r->state.load() != RS_PENDING) return false;
  if (!r->is_send) {
    for (auto it = posted_.begin(); it != posted_.end(); ++it)
      if (*it == r) {
        posted_.erase(it);
        r->st.cancelled = true;
        finish_req(r, RS_CANCELLED);
        return true;
      }
    return false;
  }
  auto& q = sendq_[r->dst];
  for (auto it = q.begin(); it != q.end(); ++it)
    if (*it == r && !r->header_posted) {
      q.erase(it);
      r->st.cancelled = true;
      finish_req(r, RS_CANCELLED);
      return true;
    }
  return false;
}

bool Engine::iprobe(int src, int tag, int ctx, Status* st) {
  std::lock_guard<std::mutex> g(mu_);
  Req probe;
  probe.src = src;
  probe.tag = tag;
  probe.ctx = ctx;
  for (auto& in : unexpected_) {
    if (match(in->hdr, probe)) {
      if (st) {
        st->source = in->hdr.src;
        st->tag = in->hdr.tag;
        st->count = in->hdr.nbytes;
        st->error = 0;
        st->cancelled = false;
      }
      return true;
    }
  }
  return false;
}

void Engine::probe(int src, int tag, int ctx, Status* st) {
  int spins = 0;
  const double tmo = wait_timeout_s();
  const auto t0 = std::chrono::steady_clock::now();
  while (!iprobe(src, tag, ctx, st)) {
    if (++spins < 1000) {
      _mm_pause();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(10));
      if (tmo > 0 && (spins & 1023) == 0 &&
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > tmo)
        throw std::runtime_error("mpit: Probe timed out after " + std::to_string(int(tmo)) +
                                 " s (source " + std::to_string(src) + ", tag " + std::to_string(tag) +
                                 "; MPIT_WAIT_TIMEOUT_S)");
    }
  }
}

// --------------------------------------------------------------------------- receive side

void Engine::deliver_locked(Incoming& in) {
  auto r = in.req;
  const Msg& h = in.hdr;
  int64_t n = h.nbytes;
  if (n > r->cap) {
    r->st.error = 15;  // ERR_TRUNCATE
    n = r->cap;
  }
  if (!in.data.empty() && n > 0) {
    if (r->rdev) {
      // host payload into HBM: the copy completes (and the request finishes, the sync-send
      // ack goes out) on the progress thread's copy poll — no stream synchronise under mu_,
      // which would stall every other message until the copy landed
      hipc(hipSetDevice(device_), "hipSetDevice");
      auto keep = std::make_shared<std::vector<uint8_t>>(std::move(in.data));
      hipc(hipMemcpyAsync(r->rbuf, keep->data(), size_t(n), hipMemcpyHostToDevice, stream_), "hipMemcpyAsync(H2D)");
      hipEvent_t ev = get_event();
      hipc(hipEventRecord(ev, stream_), "hipEventRecord");
      r->st.source = h.src;
      r->st.tag = h.tag;
      r->st.count = n;
      bytes_recv_.fetch_add(n, std::memory_order_relaxed);
      PendingCopy pc{ev, r, (h.flags & MF_SYNC) ? h.src : -1, h.aux1, [keep] {}};
      std::lock_guard<std::mutex> g(copy_mu_);
      copies_.push_back(std::move(pc));
      return;
    } else if (r->rbuf != in.data.data()) {
      std::memcpy(r->rbuf, in.data.data(), size_t(n));
    }
  }
  r->st.source = h.src;
  r->st.tag = h.tag;
  r->st.count = n;
  bytes_recv_.fetch_add(n, std::memory_order_relaxed);
  if (h.flags & MF_SYNC) {
    Msg a{};
    a.kind = MK_ACK;
    a.src = rank_;
    a.aux0 = h.aux1;
    ctrlq_[h.src].push_back(a);
  }
  finish_req(r, RS_DONE);
}

void Engine::start_dev_pull_locked(Incoming& in) {
  auto r = in.req;
  const Msg& h = in.hdr;
  int64_t n = h.nbytes;
  if (n > r->cap) {
    r->st.error = 15;
    n = r->cap;
  }
  r->st.source = h.src;
  r->st.tag = h.tag;
  r->st.count = n;
  if (device_ < 0) {
    r->err = "device message received on a rank without a device";
    finish_req(r, RS_ERROR);
    return;
  }
  hipc(hipSetDevice(device_), "hipSetDevice");
  const void* remote;
  std::string ipc_key;
  if (h.src == rank_) {
    remote = reinterpret_cast<const void*>(h.aux2);
  } else {
    hipIpcMemHandle_t hd;
    std::memcpy(&hd, h.data, sizeof(hd));
    ipc_key.assign(reinterpret_cast<const char*>(&hd), sizeof(hd));
    remote = static_cast<const uint8_t*>(open_ipc(h.src, hd, false)) + h.aux0;
  }
  if (n > 0) hipc(hipMemcpyAsync(r->rbuf, remote, size_t(n), hipMemcpyDefault, stream_), "hipMemcpyAsync(pull)");
  hipEvent_t ev = get_event();
  hipc(hipEventRecord(ev, stream_), "hipEventRecord");
  bytes_recv_.fetch_add(n, std::memory_order_relaxed);
  PendingCopy pc{ev, r, h.src, h.aux1, nullptr};
  if (!ipc_key.empty()) {
    pc.ipc_owner = h.src;
    pc.ipc_key = std::move(ipc_key);
  }
  std::lock_guard<std::mutex> g(copy_mu_);
  copies_.push_back(std::move(pc));
}

void Engine::on_header_locked(int src, const Msg& h) {
  auto in = std::make_shared<Incoming>();
  in->hdr = h;
  for (auto it = posted_.begin(); it != posted_.end(); ++it) {
    if (match(h, **it)) {
      in->req = *it;
      posted_.erase(it);
      break;
    }
  }
  if (h.kind == MK_EAGER) {
    in->data.assign(h.data, h.data + h.nbytes);
    in->got = h.nbytes;
    in->complete = true;
    if (in->req) deliver_locked(*in);
    else unexpected_.push_back(in);
  } else if (h.kind == MK_BULK) {
    in->got = 0;
    const bool direct = in->req && !in->req->rdev && in->req->cap >= h.nbytes;
    if (!direct) in->data.resize(size_t(h.nbytes));
    streaming_[src] = in;
    if (!in->req) unexpected_.push_back(in);
  } else if (h.kind == MK_DEV) {
    in->complete = true;  // payload stays in the sender's HBM until pulled
    if (in->req) start_dev_pull_locked(*in);
    else unexpected_.push_back(in);
  }
}

bool Engine::progress_recvs_locked() {
  bool did = false;
  for (int s = 0; s < world_; ++s) {
    // continue an in-flight bulk payload first (per-source FIFO order)
    if (auto in = streaming_[s]) {
      uint8_t* dst;
      const bool direct = in->req && in->data.empty();
      dst = direct ? in->req->rbuf : in->data.data();
      const int64_t m = bulk_read(s, dst + in->got, in->hdr.nbytes - in->got);
      if (m > 0) did = true;
      in->got += m;
      if (in->got == in->hdr.nbytes) {
        in->complete = true;
        streaming_[s].reset();
        if (in->req) deliver_locked(*in);
      } else {
        continue;  // do not read further headers from s until this payload is done
      }
    }
    Ring* ring = seg_->ring(s, rank_);
    uint64_t tail = ring->tail.load(std::memory_order_relaxed);
    const uint64_t head = ring->head.load(std::memory_order_acquire);
    while (tail < head) {
      Msg m = ring->slots[tail % kRingSlots];
      ++tail;
      ring->tail.store(tail, std::memory_order_release);
      did = true;
      if (m.kind == MK_ACK) {
        auto it = await_ack_.find(m.aux0);
        if (it != await_ack_.end()) {
          finish_req(it->second, RS_DONE);
          await_ack_.erase(it);
        }
        continue;
      }
      if (m.kind == MK_AM) {
        // handlers run outside mu_ (they may send); stash them
        // no handler yet (the target registers it after a collective setup step the
        // sender may have left earlier): park it until register_am
        std::lock_guard<std::mutex> g(am_mu_);
        if (am_.count(m.tag)) pending_am_.push_back(m);
        else orphan_am_.push_back(m);
        continue;
      }
      on_header_locked(s, m);
      if (streaming_[s]) break;  // payload follows; read it before any later header
    }
  }
  return did;
}

// --------------------------------------------------------------------------- send side

bool Engine::progress_sends_locked() {
  bool did = false;
  for (int d = 0; d < world_; ++d) {
    auto& cq = ctrlq_[d];
    while (!cq.empty()) {
      if (!push_msg_locked(d, cq.front())) break;
      cq.pop_front();
      did = true;
    }
    auto& q = sendq_[d];
    while (!q.empty()) {
      auto r = q.front();
      if (!r->header_posted) {
        Msg m{};
        m.tag = r->tag;
        m.ctx = r->ctx;
        m.src = rank_;
        m.nbytes = r->nbytes;
        m.seq = send_seq_[d];
        m.flags = r->sync ? MF_SYNC : 0;
        m.aux1 = r->id;
        if (r->sdev) {
          m.kind = MK_DEV;
          m.dev = r->sdevice;
          m.aux2 = int64_t(reinterpret_cast<uintptr_t>(r->sbuf));
          if (d != rank_ && r->nbytes > 0) {
            hipIpcMemHandle_t hd;
            int64_t off = 0;
            hipc(hipSetDevice(device_), "hipSetDevice");
            export_cached(r->sbuf, &hd, &off);
            std::memcpy(m.data, &hd, sizeof(hd));
            m.aux0 = off;
          }
        } else if (r->nbytes <= kInline) {
          m.kind = MK_EAGER;
          if (r->nbytes > 0) std::memcpy(m.data, r->sbuf, size_t(r->nbytes));
        } else {
          m.kind = MK_BULK;
        }
        if (!push_msg_locked(d, m)) break;
        ++send_seq_[d];
        r->header_posted = true;
        did = true;
        if (m.kind == MK_DEV) {
          await_ack_[r->id] = r;  // completes when the receiver has pulled the data
          bytes_sent_.fetch_add(r->nbytes, std::memory_order_relaxed);
          q.pop_front();
          continue;
        }
        if (m.kind == MK_EAGER) {
          bytes_sent_.fetch_add(r->nbytes, std::memory_order_relaxed);
          if (r->sync) await_ack_[r->id] = r;
          else finish_req(r, RS_DONE);
          q.pop_front();
          continue;
        }
      }
      // bulk payload
      const int64_t m = bulk_write_locked(d, r->sbuf + r->sent, r->nbytes - r->sent);
      if (m > 0) did = true;
      r->sent += m;
      if (r->sent < r->nbytes) break;
      bytes_sent_.fetch_add(r->nbytes, std::memory_order_relaxed);
      if (r->sync) await_ack_[r->id] = r;
      else finish_req(r, RS_DONE);
      q.pop_front();
    }
  }
  return did;
}

// --------------------------------------------------------------------------- device copies

void Engine::track_copy(hipEvent_t ev, std::function<void()> then) {
  {
    std::lock_guard<std::mutex> g(copy_mu_);
    copies_.push_back(PendingCopy{ev, nullptr, -1, 0, std::move(then)});
  }
  kick();
}

hipEvent_t Engine::get_event() {
  {
    std::lock_guard<std::mutex> g(ev_mu_);
    if (!ev_pool_.empty()) {
      hipEvent_t e = ev_pool_.back();
      ev_pool_.pop_back();
      return e;
    }
  }
  hipEvent_t e;
  hipc(hipSetDevice(device_), "hipSetDevice");
  hipc(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  return e;
}

void Engine::put_event(hipEvent_t e) {
  std::lock_guard<std::mutex> g(ev_mu_);
  ev_pool_.push_back(e);
}

void Engine::record_event(hipEvent_t e, hipStream_t s) { hipc(hipEventRecord(e, s), "hipEventRecord"); }

bool Engine::progress_copies() {
  std::vector<PendingCopy> done;
  {
    std::lock_guard<std::mutex> g(copy_mu_);
    if (copies_.empty()) return false;
    hipSetDevice(device_);
    for (size_t i = 0; i < copies_.size();) {
      hipError_t e = hipEventQuery(copies_[i].ev);
      if (e == hipErrorNotReady) {
        ++i;
        continue;
      }
      if (e != hipSuccess) fatal(std::string("async device copy failed: ") + hipGetErrorString(e));
      done.push_back(copies_[i]);
      copies_[i] = copies_.back();
      copies_.pop_back();
    }
  }
  if (done.empty()) return false;
  for (auto& c : done) {
    put_event(c.ev);
    if (c.ipc_owner >= 0) release_ipc(c.ipc_owner, c.ipc_key);
    if (c.req) {
      std::lock_guard<std::mutex> g(mu_);
      if (c.ack_to >= 0) {
        Msg a{};
        a.kind = MK_ACK;
        a.src = rank_;
        a.aux0 = c.ack_id;
        ctrlq_[c.ack_to].push_back(a);
      }
      finish_req(c.req, RS_DONE);
    }
    if (c.then) c.then();
  }
  return true;
}

// --------------------------------------------------------------------------- progress

void Engine::check_abort() {
  Header* h = seg_->hdr();
  if (!h->abort_flag.load(std::memory_order_acquire)) return;
  const int code = h->abort_code ? h->abort_code : 1;
  if (h->abort_rank >= 0 && h->abort_rank != rank_)
    std::fprintf(stderr, "[mpit rank %d] job aborted by rank %d (code %d): %.*s\n", rank_, h->abort_rank, code,
                 kAbortMsg, h->abort_msg);
  else if (h->abort_rank < 0)
    std::fprintf(stderr, "[mpit rank %d] job aborted by a peer (code %d)\n", rank_, code);
  std::fflush(stderr);
  ::_exit(code);
}

bool Engine::progress_once() {
  bool did = false;
  check_abort();
  {
    std::lock_guard<std::mutex> g(mu_);
    did |= progress_recvs_locked();
    did |= progress_sends_locked();
  }
  std::vector<Msg> ams;
  {
    std::lock_guard<std::mutex> g(am_mu_);
    ams.swap(pending_am_);
  }
  for (auto& m : ams) {
    AmHandler h;
    {
      std::lock_guard<std::mutex> g(am_mu_);
      h = am_[m.tag];
    }
    try {
      h(m);
    } catch (const std::exception& e) {
      // a PS server that cannot apply / serve a shard would leave every client waiting
      // forever: the whole job fails now, with the reason (init.lua:168-171)
      fatal("active-message handler " + std::to_string(m.tag) + " (from rank " + std::to_string(m.src) +
            ") failed: " + e.what());
    }
    did = true;
  }
  if (device_ >= 0) did |= progress_copies();
  std::vector<std::function<bool()>> hooks;
  {
    std::lock_guard<std::mutex> g(hook_mu_);
    for (auto& kv : hooks_) hooks.push_back(kv.second);
  }
  for (auto& h : hooks) {
    try {
      did |= h();
    } catch (const std::exception& e) {
      fatal(std::string("progress hook failed: ") + e.what());
    }
  }
  return did;
}

void Engine::check_peers() {
  // Failure detector: every rank of the node publishes its pid in the segment; a peer
  // that disappeared without Finalize (crash, OOM kill) would leave everybody blocked
  // in waits forever, so the first rank to notice aborts the whole job.
  Header* h = seg_->hdr();
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) continue;
    const RankInfo& ri = h->ranks[r];
    if (ri.attached.load(std::memory_order_acquire) != 1 || ri.pid <= 0) continue;
    bool dead = ::kill(ri.pid, 0) != 0 && errno == ESRCH;
    if (!dead) {  // an exited but not yet reaped process is a zombie: dead as well
      char path[64], buf[256] = {0};
      std::snprintf(path, sizeof(path), "/proc/%d/stat", ri.pid);
      if (FILE* f = std::fopen(path, "r")) {
        const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
        std::fclose(f);
        const char* rp = static_cast<const char*>(std::memchr(buf, ')', n));
        if (rp && rp + 2 < buf + n && rp[2] == 'Z') dead = true;
      }
    }
    if (dead) {
      std::fprintf(stderr, "[mpit rank %d] peer rank %d (pid %d) died; aborting the job\n", rank_, r, ri.pid);
      std::fflush(stderr);
      publish_abort("rank " + std::to_string(r) + " (pid " + std::to_string(ri.pid) + ") died", 70);
      ::_exit(70);
    }
  }
}

void Engine::ring(int r) {
  RankInfo& ri = seg_->hdr()->ranks[r];
  // seq_cst pairs with park(): either the sleeper sees the producer's data on its final
  // re-check, or the producer sees `sleeping` and wakes it
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (ri.sleeping.load(std::memory_order_seq_cst)) {
    ri.doorbell.fetch_add(1, std::memory_order_seq_cst);
    futex_wake_all(&ri.doorbell, true);
  }
}

void Engine::kick() {
  activity_.fetch_add(1, std::memory_order_seq_cst);
  ring(rank_);
}

bool Engine::idle_deep_ok() {
  // parking on the doorbell is safe only when every pending event is one a producer
  // rings for: nothing of ours waits on a GPU event, a full ring / bulk stream or a
  // half-read payload, and no AM is queued
  if (gpu_pending_.load(std::memory_order_acquire) > 0) return false;
  {
    std::lock_guard<std::mutex> g(copy_mu_);
    if (!copies_.empty()) return false;
  }
  {
    std::lock_guard<std::mutex> g(am_mu_);
    if (!pending_am_.empty()) return false;
  }
  std::lock_guard<std::mutex> g(mu_);
  for (int d = 0; d < world_; ++d)
    if (!sendq_[d].empty() || !ctrlq_[d].empty() || streaming_[d]) return false;
  return true;
}

void Engine::park(int64_t timeout_us, uint64_t last_act) {
  RankInfo& ri = seg_->hdr()->ranks[rank_];
  const uint32_t v = ri.doorbell.load(std::memory_order_seq_cst);
  ri.sleeping.store(1, std::memory_order_seq_cst);
  std::atomic_thread_fence(std::memory_order_seq_cst);
  // final re-check after announcing: local activity since the idle check (a kick() between
  // idle_deep_ok() and the store above saw sleeping == 0 and rang nobody: its seq_cst
  // fetch_add on activity_ precedes its fence, so it is visible here), incoming headers /
  // bulk bytes, abort
  bool work = activity_.load(std::memory_order_seq_cst) != last_act ||
              seg_->hdr()->abort_flag.load(std::memory_order_seq_cst) != 0 || !running_.load();
  for (int s = 0; s < world_ && !work; ++s) {
    Ring* rg = seg_->ring(s, rank_);
    BulkHdr* b = seg_->bulk(s, rank_);
    work = rg->head.load(std::memory_order_seq_cst) != rg->tail.load(std::memory_order_relaxed) ||
           b->wpos.load(std::memory_order_seq_cst) != b->rpos.load(std::memory_order_relaxed);
  }
  if (!work) futex_wait(&ri.doorbell, v, timeout_us, true);
  ri.sleeping.store(0, std::memory_order_relaxed);
}

void Engine::progress_loop() {
  if (device_ >= 0) hipSetDevice(device_);
  // 1 us timer slack: the idle back-off sleeps 20 us, and with the default 50 us slack each
  // wake-up (gated push -> server apply -> completion -> reply) can overshoot to ~70 us,
  // time the GPU idles at every step boundary of a parameter-server step
  // (MPIT_TIMER_SLACK_NS overrides; 0 keeps the default)
  {
    const char* e = std::getenv("MPIT_TIMER_SLACK_NS");
    const long ns = e ? std::atol(e) : 1000L;
    if (ns > 0) prctl(PR_SET_TIMERSLACK, static_cast<unsigned long>(ns), 0, 0, 0);
  }
  // Idle back-off: 256 pauses, then MPIT_PROGRESS_YIELDS yields (default 64), then either
  // a 20 us sleep (something only polling can see completes: a GPU event, a full ring) or
  // a park on this rank's futex doorbell until a producer rings it (<= 50 ms, so the peer
  // check still runs). Round 2 spun up to 4096 yields per idle period: with 8+ ranks on a
  // CPU quota the spinning threads themselves ate the quota (throttling) — parked threads
  // cost nothing.
  int idle = 0;
  uint64_t last_act = 0;
  auto last_check = std::chrono::steady_clock::now();
  int yields = 64;
  if (const char* e = std::getenv("MPIT_PROGRESS_YIELDS")) yields = std::max(0, std::atoi(e));
  const bool deep = std::getenv("MPIT_PROGRESS_PARK") == nullptr || std::atoi(std::getenv("MPIT_PROGRESS_PARK")) != 0;
  while (running_.load(std::memory_order_relaxed)) {
    const auto now = std::chrono::steady_clock::now();
    if (now - last_check > std::chrono::milliseconds(500)) {
      last_check = now;
      check_peers();
    }
    bool did = false;
    try {
      did = progress_once();
    } catch (const std::exception& e) {
      fatal(std::string("progress error: ") + e.what());
    }
    const uint64_t act = activity_.load(std::memory_order_relaxed);
    if (did || act != last_act) {
      idle = 0;
      last_act = act;
    } else if (++idle < 256) {
      _mm_pause();
    } else if (idle < 256 + yields) {
      std::this_thread::yield();
    } else if (deep && idle_deep_ok()) {
      park(50000, last_act);
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
}

// --------------------------------------------------------------------------- AM / hooks

void Engine::register_am(int id, AmHandler h) {
  std::lock_guard<std::mutex> g(am_mu_);
  am_[id] = std::move(h);
  for (auto it = orphan_am_.begin(); it != orphan_am_.end();) {
    if (it->tag == id) {
      pending_am_.push_back(*it);
      it = orphan_am_.erase(it);
    } else {
      ++it;
    }
  }
  kick();
}

void Engine::send_am(int dst, int id, const void* payload, int64_t n, int64_t aux0, int64_t aux1, int64_t aux2) {
  if (n > kInline) throw std::invalid_argument("mpit: active-message payload > 64 bytes");
  Msg m{};
  m.kind = MK_AM;
  m.tag = id;
  m.src = rank_;
  m.nbytes = n;
  m.aux0 = aux0;
  m.aux1 = aux1;
  m.aux2 = aux2;
  if (n > 0) std::memcpy(m.data, payload, size_t(n));
  {
    std::lock_guard<std::mutex> g(mu_);
    ctrlq_[dst].push_back(m);
  }
  kick();
}

int Engine::add_hook(std::function<bool()> h) {
  std::lock_guard<std::mutex> g(hook_mu_);
  int id = next_hook_++;
  hooks_[id] = std::move(h);
  return id;
}

void Engine::remove_hook(int id) {
  std::lock_guard<std::mutex> g(hook_mu_);
  hooks_.erase(id);
}

// --------------------------------------------------------------------------- collectives

void Engine::barrier() {
  Header* h = seg_->hdr();
  const uint64_t gen = h->bar_gen.load(std::memory_order_acquire);
  if (h->bar_count.fetch_add(1, std::memory_order_acq_rel) + 1 == uint64_t(world_)) {
    h->bar_count.store(0, std::memory_order_relaxed);
    h->bar_gen.fetch_add(1, std::memory_order_acq_rel);
  } else {
    int spins = 0;
    const double tmo = wait_timeout_s();
    const auto t0 = std::chrono::steady_clock::now();
    while (h->bar_gen.load(std::memory_order_acquire) == gen) {
      check_abort();
      if (++spins < 2000) {
        _mm_pause();
      } else if (spins < 2256) {
        std::this_thread::yield();
      } else {
        std::this_thread::sleep_for(std::chrono::microseconds(20));
        if (tmo > 0 && (spins & 255) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > tmo)
          fatal("barrier timed out after " + std::to_string(int(tmo)) + " s (" +
                std::to_string(h->bar_count.load()) + " of " + std::to_string(world_) +
                " ranks arrived; MPIT_WAIT_TIMEOUT_S)");
      }
    }
  }
}

std::vector<std::string> Engine::allgather_small(const std::string& blob) {
  if (int64_t(blob.size()) > kXchgBytes - 8) throw std::invalid_argument("mpit: allgather_small blob too large");
  uint8_t* mine = seg_->xchg(rank_);
  const int64_t n = int64_t(blob.size());
  std::memcpy(mine, &n, 8);
  std::memcpy(mine + 8, blob.data(), blob.size());
  std::atomic_thread_fence(std::memory_order_release);
  barrier();
  std::vector<std::string> out(world_);
  for (int r = 0; r < world_; ++r) {
    const uint8_t* p = seg_->xchg(r);
    int64_t m;
    std::memcpy(&m, p, 8);
    out[r].assign(reinterpret_cast<const char*>(p + 8), size_t(m));
  }
  barrier();
  return out;
}

void Engine::publish_abort(const std::string& why, int code) {
  // the reason goes in before the flag (release), so a peer that sees the flag reads a
  // complete message; if another rank failed first its reason is kept
  Header* h = seg_->hdr();
  if (h->abort_flag.load(std::memory_order_acquire) == 0) {
    h->abort_code = code;
    h->abort_rank = rank_;
    std::snprintf(h->abort_msg, kAbortMsg, "%s", why.c_str());
    h->abort_flag.store(1, std::memory_order_seq_cst);
  }
  for (int r = 0; r < world_; ++r) ring(r);
}

void Engine::abort(int code) {
  char why[64];
  std::snprintf(why, sizeof(why), "MPI_Abort(%d)", code);
  publish_abort(why, code ? code : 1);
  std::fprintf(stderr, "[mpit rank %d] Abort(%d)\n", rank_, code);
  std::fflush(stderr);
  ::_exit(code ? code : 1);
}

void Engine::fatal(const std::string& why, int code) {
  publish_abort(why, code);
  std::fprintf(stderr, "[mpit rank %d] fatal: %s\n", rank_, why.c_str());
  std::fflush(stderr);
  ::_exit(code);
}

}  // namespace mpit
