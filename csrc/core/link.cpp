#include "link.h"

#include <dlfcn.h>

#include <algorithm>
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

}  // namespace

PsLink::PsLink(Engine& eng, int ps_id, std::vector<int> servers, std::vector<int> clients, bool device)
    : eng_(eng),
      ps_id_(ps_id),
      servers_(std::move(servers)),
      clients_(std::move(clients)),
      device_(device),
      ctx_((1 << 26) + ps_id) {
  if (device_ && eng_.device() < 0) throw std::invalid_argument("mpit: device PS link on a rank without a device");
  if (!device_) hook_ = eng_.add_hook([this] { return poll(); });
}

PsLink::~PsLink() {
  if (hook_ >= 0) eng_.remove_hook(hook_);
  if (!comms_.empty()) {
    hipSetDevice(eng_.device());
    for (auto& kv : comms_) rccl().comm_destroy(static_cast<ncclComm_t>(kv.second));
  }
}

std::vector<std::pair<int, std::string>> PsLink::make_ids() {
  std::vector<std::pair<int, std::string>> out;
  if (!device_) return out;
  const int me = eng_.rank();
  if (std::find(servers_.begin(), servers_.end(), me) == servers_.end()) return out;
  for (int c : clients_) {
    if (c == me) continue;  // the co-located worker is served by the local fused kernel
    ncclUniqueId id;
    nccl_check(rccl().get_unique_id(&id), "ncclGetUniqueId");
    out.emplace_back(c, std::string(id.internal, sizeof(id.internal)));
  }
  return out;
}

void PsLink::connect(const std::vector<std::tuple<int, int, std::string>>& ids) {
  if (!device_) return;
  const int me = eng_.rank();
  std::vector<std::tuple<int, int, ncclUniqueId>> mine;
  for (const auto& [s, c, blob] : ids) {
    if (s != me && c != me) continue;
    if (blob.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("mpit: bad RCCL unique id");
    ncclUniqueId id;
    std::memcpy(id.internal, blob.data(), sizeof(id.internal));
    mine.emplace_back(s, c, id);
  }
  hipl(hipSetDevice(eng_.device()), "hipSetDevice");
  // every communicator of this rank in one group: a rank in several pairs must not block in
  // one pair's initialisation while its partner in another pair waits for it
  nccl_check(rccl().group_start(), "ncclGroupStart");
  std::vector<std::pair<std::pair<int, int>, ncclComm_t>> made(mine.size());
  for (size_t i = 0; i < mine.size(); ++i) {
    auto& [s, c, id] = mine[i];
    made[i].first = {s, c};
    nccl_check(rccl().comm_init_rank(&made[i].second, 2, id, s == me ? 0 : 1), "ncclCommInitRank");
  }
  nccl_check(rccl().group_end(), "ncclGroupEnd");
  for (auto& [key, comm] : made) comms_[key] = comm;
}

void* PsLink::comm_of(int peer, bool as_server) const {
  const int me = eng_.rank();
  auto it = comms_.find(as_server ? std::make_pair(me, peer) : std::make_pair(peer, me));
  if (it == comms_.end())
    throw std::runtime_error("mpit: no RCCL link between rank " + std::to_string(me) + " and rank " +
                             std::to_string(peer) + " (ps " + std::to_string(ps_id_) + ")");
  return it->second;
}

void PsLink::send(int peer, bool as_server, const void* buf, int64_t bytes, hipStream_t s) {
  if (bytes <= 0) return;
  bytes_sent_ += bytes;
  if (device_) {
    nccl_check(rccl().send(buf, size_t(bytes), ncclUint8, as_server ? 1 : 0, static_cast<ncclComm_t>(comm_of(peer, as_server)), s),
               "ncclSend");
    return;
  }
  const int64_t id = eng_.isend(buf, bytes, false, peer, tag_of(as_server), ctx_, false);
  std::lock_guard<std::mutex> g(mu_);
  q_[{peer, as_server}].push_back(Item{id, nullptr});
}

void PsLink::recv(int peer, bool as_server, void* buf, int64_t bytes, hipStream_t s) {
  if (bytes <= 0) return;
  bytes_recv_ += bytes;
  if (device_) {
    nccl_check(rccl().recv(buf, size_t(bytes), ncclUint8, as_server ? 1 : 0, static_cast<ncclComm_t>(comm_of(peer, as_server)), s),
               "ncclRecv");
    return;
  }
  const int64_t id = eng_.irecv(buf, bytes, false, peer, tag_of(!as_server), ctx_);
  std::lock_guard<std::mutex> g(mu_);
  q_[{peer, as_server}].push_back(Item{id, nullptr});
}

void PsLink::then(int peer, bool as_server, hipStream_t s, std::function<void()> f) {
  if (device_) {
    hipEvent_t ev = eng_.get_event();
    Engine::record_event(ev, s);
    eng_.track_copy(ev, std::move(f));
    return;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    q_[{peer, as_server}].push_back(Item{-1, std::move(f)});
  }
  eng_.kick();
}

bool PsLink::poll() {
  bool did = false;
  for (;;) {
    std::function<void()> run;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& kv : q_) {
        auto& q = kv.second;
        while (!q.empty() && q.front().req >= 0) {
          Status st;
          if (!eng_.test(q.front().req, &st)) break;
          if (st.error) throw std::runtime_error("mpit: PS link transfer failed");
          q.pop_front();
          did = true;
        }
        if (!q.empty() && q.front().req < 0) {
          run = std::move(q.front().f);
          q.pop_front();
          break;
        }
      }
    }
    if (!run) break;
    run();  // may queue more transfers / continuations (lock released)
    did = true;
  }
  return did;
}

}  // namespace mpit
