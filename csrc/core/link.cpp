#include "link.h"

#include <dlfcn.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include <rccl/rccl.h>

namespace mpit {

namespace {

// RCCL resolved at run time from the copy already in the process (PyTorch's, the one
// torch.distributed's "nccl" backend uses), else ROCm's: one RCCL per process, and no
// link-time dependency of the module on a library that only datapath 3 needs.
struct Rccl {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = nullptr;
    for (const char* name : {"librccl.so", "librccl.so.1"})
      if ((h = ::dlopen(name, RTLD_NOW | RTLD_NOLOAD))) break;
    if (!h) h = ::dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) throw std::runtime_error(std::string("mpit: datapath 3 needs RCCL: ") + ::dlerror());
    auto sym = [h](const char* n) {
      void* p = ::dlsym(h, n);
      if (!p) throw std::runtime_error(std::string("mpit: RCCL symbol missing: ") + n);
      return p;
    };
    x.get_unique_id = reinterpret_cast<decltype(x.get_unique_id)>(sym("ncclGetUniqueId"));
    x.comm_init_rank = reinterpret_cast<decltype(x.comm_init_rank)>(sym("ncclCommInitRank"));
    x.comm_destroy = reinterpret_cast<decltype(x.comm_destroy)>(sym("ncclCommDestroy"));
    x.send = reinterpret_cast<decltype(x.send)>(sym("ncclSend"));
    x.recv = reinterpret_cast<decltype(x.recv)>(sym("ncclRecv"));
    x.group_start = reinterpret_cast<decltype(x.group_start)>(sym("ncclGroupStart"));
    x.group_end = reinterpret_cast<decltype(x.group_end)>(sym("ncclGroupEnd"));
    x.error_string = reinterpret_cast<decltype(x.error_string)>(sym("ncclGetErrorString"));
    return x;
  }();
  return r;
}

void nccl_check(ncclResult_t e, const char* what) {
  if (e != ncclSuccess) throw std::runtime_error(std::string("mpit link RCCL error in ") + what + ": " + rccl().error_string(e));
}

void hipl(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("mpit link HIP error in ") + what + ": " + hipGetErrorString(e));
}

bool env_on(const char* n) {
  const char* e = std::getenv(n);
  return e && std::atoi(e) != 0;
}

// the sequencer's notice of one transfer (AM payload, <= 64 bytes)
struct Notice {
  int64_t xid;    // the server's id of the transfer
  int64_t coff;   // client buffer byte offset
  int64_t bytes;
  int32_t server, client;
  int32_t to_client, window;
};
static_assert(sizeof(Notice) <= 64, "notice must fit an active message");

}  // namespace

PsLink::PsLink(Engine& eng, int ps_id, std::vector<int> members, bool device)
    : eng_(eng), ps_id_(ps_id), members_(std::move(members)), device_(device), ctx_((1 << 26) + ps_id) {
  if (members_.empty()) throw std::invalid_argument("mpit: PS link without members");
  if (device_ && eng_.device() < 0) throw std::invalid_argument("mpit: device PS link on a rank without a device");
  legacy_ = !device_ && env_on("MPIT_LINK_LEGACY");
  rdv_ = !device_ && env_on("MPIT_LINK_RDV");
  if (const char* e = std::getenv("MPIT_LINK_JITTER_US")) jitter_us_ = std::max(0, std::atoi(e));
  rng_.seed(uint32_t(eng_.rank() * 7919 + ps_id * 104729 + (std::getenv("MPIT_LINK_SEED") ? std::atoi(std::getenv("MPIT_LINK_SEED")) : 0)));
  if (device_) {
    hipl(hipSetDevice(eng_.device()), "hipSetDevice");
    int lo = 0, hi = 0;
    hipl(hipDeviceGetStreamPriorityRange(&lo, &hi), "priority range");
    hipl(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "link stream");
  }
  eng_.register_am(am_req(), [this](const Msg& m) { on_req(m); });
  eng_.register_am(am_post(), [this](const Msg& m) { on_post(m); });
  eng_.register_am(am_cts(), [this](const Msg& m) {
    std::lock_guard<std::mutex> g(mu_);
    ++cts_got_[m.src];
  });
  hook_ = eng_.add_hook([this] { return poll(); });
}

PsLink::~PsLink() {
  if (hook_ >= 0) eng_.remove_hook(hook_);
  for (int id : {am_req(), am_post(), am_cts()}) eng_.register_am(id, [](const Msg&) {});
  if (device_) {
    hipSetDevice(eng_.device());
    if (stream_) hipStreamSynchronize(stream_);
    if (comm_) rccl().comm_destroy(static_cast<ncclComm_t>(comm_));
    if (stream_) hipStreamDestroy(stream_);
  }
}

int PsLink::index_of(int world_rank) const {
  for (size_t i = 0; i < members_.size(); ++i)
    if (members_[i] == world_rank) return int(i);
  throw std::invalid_argument("mpit: rank " + std::to_string(world_rank) + " is not a member of PS " + std::to_string(ps_id_));
}

std::string PsLink::make_id() {
  if (!device_ || eng_.rank() != sequencer()) return {};
  ncclUniqueId id;
  nccl_check(rccl().get_unique_id(&id), "ncclGetUniqueId");
  return std::string(id.internal, sizeof(id.internal));
}

void PsLink::connect(const std::string& blob) {
  if (!device_) return;
  if (blob.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("mpit: bad RCCL unique id");
  ncclUniqueId id;
  std::memcpy(id.internal, blob.data(), sizeof(id.internal));
  hipl(hipSetDevice(eng_.device()), "hipSetDevice");
  ncclComm_t c = nullptr;
  nccl_check(rccl().comm_init_rank(&c, int(members_.size()), id, index_of(eng_.rank())), "ncclCommInitRank");
  comm_ = c;
}

void PsLink::jitter() {
  if (jitter_us_ <= 0) return;
  std::uniform_int_distribution<int> d(0, jitter_us_);
  const int us = d(rng_);
  if (us > jitter_us_ / 2) ::usleep(useconds_t(us));
}

// ------------------------------------------------------------------------------ ordering

void PsLink::order(int client, bool to_client, int window, int64_t coff, int64_t bytes, std::function<void()> at_server) {
  if (legacy_) {  // pre-sequencer layout (test only): the server queues its side at once
    at_server();
    return;
  }
  Notice n{};
  {
    std::lock_guard<std::mutex> g(mu_);
    n.xid = next_xid_++;
    at_server_[n.xid] = std::move(at_server);
  }
  n.coff = coff;
  n.bytes = bytes;
  n.server = eng_.rank();
  n.client = client;
  n.to_client = to_client ? 1 : 0;
  n.window = window;
  jitter();
  eng_.send_am(sequencer(), am_req(), &n, sizeof(n));
}

void PsLink::set_client(ClientFn at_client) {
  std::lock_guard<std::mutex> g(mu_);
  at_client_ = std::move(at_client);
}

// sequencer: the arrival order of requests here IS the global order; the notices go out to
// both endpoints in it (one FIFO control ring from here to each rank)
void PsLink::on_req(const Msg& m) {
  if (eng_.rank() != sequencer()) throw std::runtime_error("mpit: PS link request at a rank that is not the sequencer");
  Notice n;
  std::memcpy(&n, m.data, sizeof(n));
  ++ordered_;
  eng_.send_am(n.server, am_post(), &n, sizeof(n), 0);
  if (n.client != n.server) eng_.send_am(n.client, am_post(), &n, sizeof(n), 1);
}

bool PsLink::self_mode() {
  static const bool on = env_on("MPIT_LINK_SELF");
  return on;
}

// self-loop: queue the client's side of the armed notice right behind the server's op (the
// two then go out in one RCCL group: a send to self needs its receive in the same group)
void PsLink::self_join() {
  if (!self_armed_) return;
  self_armed_ = false;
  ClientFn c;
  {
    std::lock_guard<std::mutex> g(mu_);
    c = at_client_;
  }
  if (!c) throw std::runtime_error("mpit: PS link self-loop notice without a client");
  c(eng_.rank(), self_to_client_, self_window_, self_coff_, self_bytes_);
}

void PsLink::on_post(const Msg& m) {
  Notice n;
  std::memcpy(&n, m.data, sizeof(n));
  jitter();
  const bool as_client = m.aux0 == 1;
  if (!as_client) {
    std::function<void()> f;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = at_server_.find(n.xid);
      if (it == at_server_.end()) throw std::runtime_error("mpit: PS link notice for an unknown transfer");
      f = std::move(it->second);
      at_server_.erase(it);
    }
    if (n.client == n.server) {  // self-loop (the sequencer sent this rank one notice)
      self_armed_ = true;
      self_coff_ = n.coff;
      self_bytes_ = n.bytes;
      self_window_ = n.window;
      self_to_client_ = n.to_client != 0;
    }
    f();
    if (self_armed_) throw std::runtime_error("mpit: PS link self-loop transfer queued no server side");
  } else {
    ClientFn c;
    {
      std::lock_guard<std::mutex> g(mu_);
      c = at_client_;
    }
    if (!c) throw std::runtime_error("mpit: PS link notice for a client that has no link buffers");
    c(n.server, n.to_client != 0, n.window, n.coff, n.bytes);
  }
}

// ------------------------------------------------------------------------------ data ops

void PsLink::send(int peer, const void* buf, int64_t bytes, hipEvent_t after) {
  if (bytes <= 0) return;
  bytes_sent_ += bytes;
  if (device_) {
    if (after) {
      flush_group();
      hipl(hipStreamWaitEvent(stream_, after, 0), "link waits local work");
    }
    batch_.push_back({true, peer, const_cast<void*>(buf), bytes});
    if (peer == eng_.rank()) self_join();
    return;
  }
  Op o{kSend};
  o.peer = peer;
  o.sbuf = buf;
  o.bytes = bytes;
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(std::move(o));
  }
  if (peer == eng_.rank()) self_join();
}

void PsLink::recv(int peer, void* buf, int64_t bytes, hipEvent_t after) {
  if (bytes <= 0) return;
  bytes_recv_ += bytes;
  if (device_) {
    if (after) {
      flush_group();
      hipl(hipStreamWaitEvent(stream_, after, 0), "link waits local work");
    }
    batch_.push_back({false, peer, buf, bytes});
    if (peer == eng_.rank()) self_join();
    return;
  }
  Op o{kRecv};
  o.peer = peer;
  o.rbuf = buf;
  o.bytes = bytes;
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(std::move(o));
  }
  if (peer == eng_.rank()) self_join();
}

void PsLink::then(std::function<void()> f) {
  if (device_) {
    if (!batch_.empty()) {
      batch_then_.push_back(std::move(f));  // after the group the pending ops go out in
      return;
    }
    hipEvent_t ev = eng_.get_event();
    Engine::record_event(ev, stream_);
    eng_.track_copy(ev, std::move(f));
    return;
  }
  call(std::move(f));
}

void PsLink::call(std::function<void()> f) {
  if (device_) {
    f();
    return;
  }
  Op o{kCall};
  o.f = std::move(f);
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(std::move(o));
  }
  eng_.kick();
}

void PsLink::record(hipEvent_t e) {
  if (!device_) return;
  flush_group();
  hipl(hipEventRecord(e, stream_), "link record");
}

void PsLink::flush_group() {
  if (!device_ || batch_.empty()) return;
  hipl(hipSetDevice(eng_.device()), "hipSetDevice");
  auto* c = static_cast<ncclComm_t>(comm_);
  if (!c) throw std::runtime_error("mpit: PS link used before connect()");
  nccl_check(rccl().group_start(), "ncclGroupStart");
  for (const auto& o : batch_) {
    const int pr = index_of(o.peer);
    if (o.send) nccl_check(rccl().send(o.buf, size_t(o.bytes), ncclUint8, pr, c, stream_), "ncclSend");
    else nccl_check(rccl().recv(o.buf, size_t(o.bytes), ncclUint8, pr, c, stream_), "ncclRecv");
  }
  nccl_check(rccl().group_end(), "ncclGroupEnd");
  ++groups_;
  batch_.clear();
  std::vector<std::function<void()>> fs;
  fs.swap(batch_then_);
  if (!fs.empty()) {
    hipEvent_t ev = eng_.get_event();
    Engine::record_event(ev, stream_);
    eng_.track_copy(ev, [fs] {
      for (auto& f : fs) f();
    });
  }
}

// host self-loop: the head op is one half of a send / receive pair to this rank itself
// (queued back to back, like the device path's one RCCL group): the other half starts too,
// or the head would wait forever for an op queued behind it. (mu_ held)
void PsLink::start_self_partner() {
  if (q_.size() < 2) return;
  Op& h = q_[0];
  Op& o = q_[1];
  if (h.peer != eng_.rank() || o.peer != eng_.rank() || o.req >= 0 || o.kind == kCall || o.kind == h.kind) return;
  o.req = o.kind == kSend ? eng_.isend(o.sbuf, o.bytes, false, o.peer, 1, ctx_, false)
                          : eng_.irecv(o.rbuf, o.bytes, false, o.peer, 1, ctx_);
}

// host: the FIFO as a stream. The head op starts when everything before it is done.
bool PsLink::poll() {
  if (device_) {
    const bool did = !batch_.empty();
    flush_group();
    return did;
  }
  bool did = false;
  for (;;) {
    std::function<void()> run;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (q_.empty()) break;
      Op& o = q_.front();
      if (o.kind == kCall) {
        run = std::move(o.f);
        q_.pop_front();
      } else if (o.kind == kSend) {
        if (o.req < 0) {
          // rendezvous: a send runs only against a receive at the head of the peer's FIFO
          // (a self-loop pair is one group: no clear-to-send between its two halves)
          const bool self = o.peer == eng_.rank();
          if (rdv_ && !self && cts_got_[o.peer] <= cts_used_[o.peer]) break;
          if (rdv_ && !self) ++cts_used_[o.peer];
          o.req = eng_.isend(o.sbuf, o.bytes, false, o.peer, 1, ctx_, false);
        }
        Status st;
        if (!eng_.test(o.req, &st)) {
          start_self_partner();
          break;
        }
        if (st.error) throw std::runtime_error("mpit: PS link send failed");
        q_.pop_front();
        did = true;
        continue;
      } else {
        if (o.req < 0) {
          o.req = eng_.irecv(o.rbuf, o.bytes, false, o.peer, 1, ctx_);
          if (rdv_ && o.peer != eng_.rank()) eng_.send_am(o.peer, am_cts(), nullptr, 0);
        }
        Status st;
        if (!eng_.test(o.req, &st)) {
          start_self_partner();
          break;
        }
        if (st.error) throw std::runtime_error("mpit: PS link receive failed");
        q_.pop_front();
        did = true;
        continue;
      }
    }
    run();  // local work / continuation (may queue more ops; lock released)
    did = true;
  }
  return did;
}

}  // namespace mpit
