// Native parameter server and client (SURVEY §2.3 P1–P5), MI355X-first.
//
// Reference behaviour kept: the eight-tag protocol (asyncsgd/init.lua:3-10), contiguous
// even sharding with the remainder on the last shard (asyncsgd/pclient.lua:116-128, here
// 0-based), parameter init pushed by the first client (asyncsgd/pclient.lua:130-133,
// asyncsgd/pserver.lua:152-158), gradient push + ack, parameter pull on request, stop
// counting (asyncsgd/pserver.lua:125-139), server-side update rules including the
// BiCNN adaptive family (BiCNN/pserver.lua:115-205).
//
// What changed and why (MI355X):
//  * Data never travels inside messages. Every client exposes two IPC windows in HBM
//    (rx: where pulled shards land, normally the model's own flat parameters; tx: the
//    pushed gradient / parameter vector). A server reads tx and writes rx directly over
//    xGMI; only 128-B control messages go through the shm rings.
//  * Datapath 2 (default on HBM): every remote client has its own high-priority "link"
//    stream and inbox/outbox pair; its gradient shard is pulled (SDMA peer copy over its
//    own xGMI link) while other clients' transfers proceed on theirs, the fused update
//    rule runs on the server stream (and snapshots the shard into the outbox when a pull
//    is due), and the snapshot is pushed back on the link stream. The worker on the
//    server's own GPU is served by ONE fused kernel (read tx, update, write rx) with no
//    copies. Datapath 0 does that fused kernel for every client, reading/writing peer
//    HBM directly; datapath 1 uses serial SDMA copies around a local kernel.
//  * All updates of a shard are serialised on that one stream, so a pull always copies a
//    consistent snapshot (the reference sends p while recvgrad mutates it,
//    asyncsgd/pserver.lua:81).
//  * Optional bounded staleness (SSP): a pull by a client more than `staleness`
//    pushes ahead of the slowest client is deferred (BASELINE config 4).
//  * Clients gate their push on a HIP event of the producing stream, so Python never
//    blocks to send; replies are counted and wait() sleeps with the GIL released.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <vector>

#include "engine.h"
#include "link.h"
#include "window.h"

namespace mpit {

enum PsTag : int {
  kTagInit = 1,
  kTagGrad = 2,
  kTagSendParam = 3,
  kTagParam = 4,
  kTagHeader = 5,
  kTagStop = 6,
  kTagParamTail = 7,
  kTagGradTail = 8,
};
// kPsWithPull (tag 2): reply with the refreshed shard; kPsFromRx (tag 4): the pushed
// parameters are in the client's fp32 rx window, not its tx window (an EASGD client whose
// wire is bf16 initialises the shards with exact fp32 weights).
// kPsGpuGate: from the co-located device client — the message was sent when issued, not when
// the client's GPU work before it finished; the server's stream waits on the client's gate
// event (PSClient::pop_gate) before serving it
enum PsFlags : int64_t { kPsWithPull = 1, kPsFromRx = 2, kPsGpuGate = 4 };

inline int ps_am_id(int ps_id, int tag) { return 4096 + ps_id * 16 + tag; }

// Server-side rule (BiCNN/plaunch.lua optimisation flags). kind: 0 = p += a*g (Downpour /
// EASGD / local-mode pushes), 1 rmsprop, 2 adam, 3 adamax, 4 adagrad, 5 adadelta.
struct ServerRule {
  int kind = 0;
  float a = 1.f;
  float lr = 0.f, decay = 0.9f, mom = 0.f, eps = 1e-8f;
  float b1 = 0.9f, b2 = 0.999f, rho = 0.95f, lrd = 0.f;
  int64_t step_div = 1;
};

struct ServerStats {
  int64_t grads = 0, pulls = 0, param_pushes = 0, deferred = 0;
  int64_t batches = 0;  // queued-update flushes (see PSServer::flush_grads)
  int64_t multi = 0;    // of them, flushes that applied >= 2 pieces in one launch
};

// A contiguous piece of a server's shard named by a message: [o, o + n) relative to the
// shard start. A client normally addresses whole shards; a client that splits one server's
// shard into several entries (bench.py --emulate-shards: K shards on one GPU) sends the
// absolute offset / length of its entry in aux1 / aux2 (tags 2, 4, 5).
struct Sub {
  int64_t o = 0, n = 0;
};

class PSClient;

class PSServer {
 public:
  // members: world ranks of the window members, in window member order; clients: the
  // world ranks of this server's clients. p / state / inbox are caller-owned memory
  // (device when device=true). state = rule-specific buffers, each shard_len fp32.
  PSServer(Engine& eng, int ps_id, Window& rx, Window& tx, std::vector<int> members, std::vector<int> clients,
           int64_t shard_off, int64_t shard_len, bool device, uintptr_t p, std::vector<uintptr_t> state,
           uintptr_t inbox, ServerRule rule, int datapath, int64_t staleness, bool grad_bf16, int init_rank);
  ~PSServer();
  // the started device server of (ps_id, rank) in this process (the co-located one)
  static PSServer* local(int ps_id, int rank);
  void start();
  bool done() const { return stopped_.load() >= int(clients_.size()); }
  void wait_done();
  ServerStats stats() const;
  int64_t version() const { return version_.load(); }
  // rule step counter and update version, saved / restored by checkpoints (quiescent server)
  int64_t step() const { return t_.load(); }
  void set_counters(int64_t step, int64_t version) {
    t_.store(step);
    version_.store(version);
  }
  void set_lr(float lr);
  void sync();  // wait for all queued server work
  // datapath 3: the instance's two-sided data plane (csrc/core/link.h); set before start()
  void set_link(PsLink* l) { link_ = l; }

 private:
  void on_msg(const Msg& m);
  Sub sub_of(const Msg& m) const;
  bool maybe_fault(int kind);
  void do_param(int c, bool from_rx, Sub sb);
  void do_grad(int c, bool pull, Sub sb);
  void do_pull(int c, Sub sb);
  void apply_rule(const void* g, void* out, Sub sb, int ci);
  std::vector<uintptr_t> rule_ptrs(const void* g, void* out, Sub sb) const;
  // gradient pieces of the direct (non-link) path that arrive in one progress sweep are
  // applied together: ONE multi-segment launch (ew_update_multi) instead of one per piece.
  // Plain apply / RMSProp only (their scalars do not change per push); a piece overlapping
  // a queued one, any other message and the end of the sweep (engine hook) flush the queue
  // in arrival order. MPIT_PS_BATCH=0 disables.
  struct PendingGrad {
    int c;
    bool pull, defer;
    Sub sb;
  };
  bool batchable(int c) const;
  void queue_grad(int c, bool pull, Sub sb);
  bool flush_grads();
  bool batch_ = true;
  std::vector<PendingGrad> pend_;
  struct FlushGate {
    std::mutex mu;
    PSServer* s = nullptr;
  };
  std::shared_ptr<FlushGate> fg_;
  int hook_ = -1;
  void copy_out(int c, Sub sb);
  // datapath 3: the shard's data with remote client c as RCCL / host messages (link.h)
  PsLink* link_ = nullptr;
  // datapath 3: a remote client's data as link messages; with the link's self-loop
  // (PsLink::self_mode) the co-located client's too
  bool messaged(int ci, int c) const {
    return datapath_ == 3 && ci >= 0 && (c != eng_.rank() || PsLink::self_mode());
  }
  void grad_msg(int c, int ci, bool pull, bool defer_pull, Sub sb);
  void pull_msg(int c, int ci, Sub sb);
  void param_msg(int c, int ci, bool from_rx, Sub sb, std::function<void()> after = nullptr);
  void reply(int c, int tag);
  // the co-located device client of rank c that takes GPU events instead of finished replies
  PSClient* early_client(int c) const;
  // replies to client c: at once with the update's event for the co-located device client,
  // else once the work queued so far on stream_ finished
  void finish_for(int c, std::function<void()> replies);
  void finish(std::function<void()> then);
  void release_deferred();
  int member_of(int world_rank) const;
  int client_index(int world_rank) const;

  Engine& eng_;
  int ps_id_;
  Window& rx_;
  Window& tx_;
  std::vector<int> members_, clients_;
  int64_t off_, len_;
  bool device_;
  void* p_;
  std::vector<void*> st_;
  void* inbox_;
  ServerRule rule_;
  std::atomic<float> lr_;  // rule_.lr, changed by set_lr from the caller's thread while the progress thread runs
  int datapath_;
  int64_t staleness_;
  bool grad_bf16_;
  hipStream_t stream_ = nullptr;
  // datapath 2 (default on HBM): one "link" stream + staging pair per client, so the
  // gradient pulls and parameter pushes of different clients run concurrently over
  // their own xGMI links (SDMA copies) and only the local fused update is serialised on
  // stream_. stage_ = [clients][inbox | outbox] of shard_len fp32 each (also datapath 3's
  // staging). MPIT_PS_LINK_STREAMS=k caps the link streams (client i uses stream i % k);
  // default 2 on a server co-located with a worker, one per client on a dedicated server.
  // The link streams carry only SDMA copies and event waits.
  std::vector<hipStream_t> cstream_;
  hipStream_t link(int ci) const { return cstream_[size_t(ci) % cstream_.size()]; }
  std::vector<hipEvent_t> ev_in_, ev_up_, ev_out_;
  uint8_t* stage_ = nullptr;
  void finish_on(hipStream_t s, std::function<void()> then);
  // the worker on this very GPU is served by the fused local kernel (no copies at all),
  // unless MPIT_PS_FORCE_PIPE=1 (the K-shard emulation: every push takes the link path)
  bool force_pipe_ = false;
  bool pipelined(int ci, int c) const {
    return device_ && datapath_ == 2 && ci >= 0 && (c != eng_.rank() || force_pipe_);
  }
  // fault injection (tests of the fail-fast path): MPIT_PS_FAULT=grad|pull|param[:N] throws
  // in the Nth such request, drop[:N] silently ignores gradient pushes from the Nth on;
  // MPIT_PS_FAULT_RANK=r limits it to the server on rank r
  int fault_kind_ = 0, fault_at_ = 1, fault_client_ = -1;
  std::atomic<int> fault_seen_{0};
  std::atomic<int> stopped_{0};
  std::atomic<int64_t> version_{0};
  int init_rank_;                 // client whose parameter push initialises the shard (-1: ready)
  int64_t init_left_;             // elements of the shard that push has still to cover
  std::vector<Msg> backlog_;      // grads / pulls that arrived before that push
  std::atomic<int64_t> t_{0};  // rule step counter (adam / adamax / adagrad / adadelta)
  std::vector<int64_t> clock_;  // pushes received per client (SSP)
  std::vector<int64_t> tpush_;  // per client: the rule step its current push took (split entries)
  std::deque<std::pair<int, Sub>> deferred_;  // pulls (client, piece) waiting for stragglers
  mutable std::mutex mu_;
  std::condition_variable cv_;
  ServerStats stats_;
};

class PSClient {
 public:
  // one entry per shard: (server rank, absolute offset, length). A server normally appears
  // once; several entries of one server split its shard (emulation of K shards).
  PSClient(Engine& eng, int ps_id, std::vector<int> servers, std::vector<int64_t> offs, std::vector<int64_t> lens);
  ~PSClient();
  void start();            // register reply handlers, send shard info (tag 1)
  void send_grad(hipStream_t s, bool with_pull);  // gated on the work queued on s
  // the same for ONE shard (server index k): pushes overlapped with the backward as soon
  // as a shard's gradients are complete
  void send_grad_to(hipStream_t s, int k, bool with_pull);
  void recv_param(hipStream_t s);  // tag 5 header -> tag 3 once the shard landed in rx;
                                   // gated on s when rx is still being read there
  void send_param(hipStream_t s, bool from_rx = false);
  void stop();
  // until every outstanding reply arrived (GIL released); raises after MPIT_PS_TIMEOUT_S
  // (default 0 = never, opt-in on every datapath) with the number of replies still missing
  void wait();
  // datapath 3: shard data as messages over `l` (link.h) from / into this client's own
  // buffers: rx (fp32 parameters, pulls land here), tx (push window, tx_es bytes / element)
  void set_link(PsLink* l, uintptr_t rx, uintptr_t tx, int tx_es);
  bool test() const { return pending_.load() == 0; }
  int64_t pending() const { return pending_.load(); }
  int64_t replies() const { return replies_.load(); }
  // Co-located server (the same rank, a device shard on the local fused path): it replies as
  // soon as its update is QUEUED and hands over the GPU event that completes it, instead of
  // replying after a host poll of that event (MPIT_PS_LOCAL_EVENTS=0: the poll). The client's
  // next GPU work must wait on those events: take_deps(s) makes stream s wait on every event
  // handed over so far (called by the Python wait / test before anything reads the shard).
  void add_gpu_dep(hipEvent_t e);
  void take_deps(hipStream_t s);
  // the gate event of the oldest kPsGpuGate message not yet served (server side)
  hipEvent_t pop_gate();
  // the client of (ps_id, rank) in this process, if it runs as a device client
  static PSClient* local(int ps_id, int rank);

 private:
  struct GateQueue;
  void gate(hipStream_t s, std::function<void()> send);
  void send_entry(int k, int tag, int64_t flags);
  void on_reply(const Msg& m);
  void local_done();
  // the entry's pull lands through the link (a completion of our own to wait for)
  int link_recvs(int k, int tag, int64_t flags) const;
  PsLink* link_ = nullptr;
  uint8_t* rx_ = nullptr;
  uint8_t* tx_ = nullptr;
  int tx_es_ = 4;
  Engine& eng_;
  std::shared_ptr<GateQueue> gq_;
  int hook_ = -1;
  int ps_id_;
  std::vector<int> servers_;
  std::vector<int64_t> offs_, lens_;
  std::atomic<int64_t> pending_{0};
  std::atomic<int64_t> replies_{0};
  std::atomic<uint32_t> reply_seq_{0};  // futex word bumped by every reply
  std::mutex dep_mu_;
  std::vector<hipEvent_t> deps_;  // update events of the co-located server not yet waited on
  std::deque<hipEvent_t> gates_;  // gate events of kPsGpuGate messages, in send order
  bool gpu_gate(int k) const;     // entry k's server is the co-located device server
  void send_local(hipStream_t s, int k, int tag, int64_t flags);
};

}  // namespace mpit
