// Two-sided point-to-point data plane of one parameter-server instance (datapath 3).
//
// The reference moves every shard as an MPI Isend / Irecv pair handed the Torch storage's
// data pointer — a device pointer under a CUDA-aware MPI (lua-mpi.h:70-78, init.lua:48,88).
// Datapaths 0-2 replace that with one-sided access: the server reads the worker's gradient
// window and writes its parameter window in HBM through IPC peer mappings. Datapath 3 keeps
// the reference's two-sided shape on MI355X: gradient shards and refreshed shards travel as
// RCCL send / recv pairs over xGMI between the worker's and the server's GPU, and no rank ever
// maps another process's allocation. It is the path for a node whose peer mappings are
// unavailable or broken (bench.py switches to it when its pre-flight check fails).
//
// Deadlock freedom, by construction:
//  * ONE RCCL communicator over the instance's members and ONE link stream per rank. Every
//    RCCL op of a rank — its client role and its server role alike — is queued on that one
//    stream by the rank's progress thread, so a rank's ops form a single total order whatever
//    the streams-to-hardware-queue mapping (GPU_MAX_HW_QUEUES) does to them.
//  * A global order over all transfers of the instance: the server that decides a transfer
//    (on a client's control message, or when an SSP-deferred pull is released) asks the
//    instance's sequencer (its lowest member rank) for it; the sequencer hands every request
//    a place in one sequence and tells BOTH endpoints, over its FIFO control rings, in that
//    sequence. Each rank queues its side of a transfer when the sequencer's notice arrives,
//    so on every rank the link ops are queued in increasing global sequence.
//  * Local GPU work queued between link ops (the server's update of a received gradient, the
//    snapshot of a pulled shard) depends only on link ops queued before it, and a client
//    sends its control message only once the data it pushes is complete (its gate event).
//  * Then the unfinished transfer with the smallest sequence number always completes: on each
//    of its two ranks every op queued ahead of it belongs to a smaller, hence finished,
//    transfer, or is local work that depends only on those. By induction every transfer
//    completes, for any interleaving of control messages and any stream-to-queue merge.
//  * Consecutive link ops queued in one progress sweep are issued as one ncclGroupStart/End,
//    so a worker's receives from its K servers progress together instead of one by one.
//
// Self-loop (MPIT_LINK_SELF=1): the sequencer's notice of a transfer between a rank's own
// server and client goes to that rank once (as server); when the server queues its side
// (send or recv to itself) the client's matching side is queued right behind it, into the
// same RCCL group, before anything flushes the batch. Same order, same events, one GPU.
//
// Without a GPU (the CPU test tier) the same ops run over the engine's tagged host messages
// in ONE FIFO per rank, processed like a stream: an op starts when the ops before it are
// done, and local work runs as a queued call. Two host modes: free (a send completes once
// the engine took its bytes) and rendezvous (MPIT_LINK_RDV=1: a send completes only after
// the receiver's matching receive reached the head of the receiver's FIFO, as a blocking
// RCCL send at the head of a hardware queue does). tests/mp/ps_link_rdv.py runs the protocol
// in rendezvous mode under randomised control-message timing (MPIT_LINK_JITTER_US), and also
// the pre-sequencer layout (MPIT_LINK_LEGACY=1: clients queue their ops when they send their
// control message, servers when it arrives), which deadlocks there.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "engine.h"

namespace mpit {

class PsLink {
 public:
  // members: world ranks of the PS instance (servers and clients), in a common order on
  // every member; device: RCCL between GPUs, else the engine's host messages
  PsLink(Engine& eng, int ps_id, std::vector<int> members, bool device);
  ~PsLink();
  PsLink(const PsLink&) = delete;
  PsLink& operator=(const PsLink&) = delete;

  bool device() const { return device_; }
  bool legacy() const { return legacy_; }
  // self-loop (MPIT_LINK_SELF=1, datapath 3 only): a rank's own client and server also move
  // their shard through the link — a grouped RCCL send / recv to itself on the link stream —
  // instead of the local fused path. This puts datapath 3's device branch (RCCL ops, link
  // stream, event hand-offs, continuations) on ONE GPU: a 1-rank job runs it end to end.
  static bool self_mode();
  int sequencer() const { return members_.front(); }
  // RCCL: the sequencer makes the communicator's unique id (128 bytes; others: empty); the
  // caller broadcasts it and every member calls connect() with it (collective)
  std::string make_id();
  void connect(const std::string& id);

  // --- ordering -----------------------------------------------------------------------
  // Server side: have a transfer between this server and client c ordered. to_client: the
  // server sends (a pulled shard), else the client does (a gradient or parameter push).
  // window / coff name the client's buffer (0 = rx, 1 = tx; byte offset). at_server runs on
  // this rank's progress thread at the transfer's turn and queues this rank's side of it.
  void order(int client, bool to_client, int window, int64_t coff, int64_t bytes, std::function<void()> at_server);
  // Client side: at_client(server, to_client, window, coff, bytes) queues the client's side
  // at the transfer's turn
  using ClientFn = std::function<void(int, bool, int, int64_t, int64_t)>;
  void set_client(ClientFn at_client);

  // --- this rank's side of a transfer (from at_server / at_client, in order) ---------------
  // device: queued on the link stream after `after` (an event of local work, or null)
  void send(int peer, const void* buf, int64_t bytes, hipEvent_t after = nullptr);
  void recv(int peer, void* buf, int64_t bytes, hipEvent_t after = nullptr);
  // f runs on the progress thread once everything queued so far has completed
  void then(std::function<void()> f);
  // device: record e on the link stream after everything queued so far (host: no-op)
  void record(hipEvent_t e);
  // host: f runs when the FIFO reaches it (local work in stream order); device: runs now
  void call(std::function<void()> f);
  hipStream_t stream() const { return stream_; }

  int64_t bytes_sent() const { return bytes_sent_; }
  int64_t bytes_recv() const { return bytes_recv_; }
  int64_t ordered() const { return ordered_; }  // transfers this rank sequenced
  int64_t groups() const { return groups_; }    // device: ncclGroup batches issued

 private:
  enum Kind { kSend = 0, kRecv = 1, kCall = 2 };
  struct Op {
    Kind kind;
    int peer = -1;
    const void* sbuf = nullptr;
    void* rbuf = nullptr;
    int64_t bytes = 0;
    std::function<void()> f;
    int64_t req = -1;  // host: engine request once started
  };
  int am_req() const { return (1 << 20) + ps_id_ * 4; }
  int am_post() const { return am_req() + 1; }
  int am_cts() const { return am_req() + 2; }
  void on_req(const Msg& m);   // sequencer
  void on_post(const Msg& m);  // endpoint
  void jitter();
  bool poll();                 // host FIFO (engine hook)
  void start_self_partner();   // host self-loop pair (mu_ held)
  void flush_group();          // device: issue the batched RCCL ops
  int index_of(int world_rank) const;

  Engine& eng_;
  int ps_id_;
  std::vector<int> members_;
  bool device_;
  bool legacy_ = false, rdv_ = false;
  int ctx_;
  void* comm_ = nullptr;  // device: ncclComm_t over members_
  hipStream_t stream_ = nullptr;
  // device: RCCL ops of the current progress sweep, issued as one group
  struct DevOp {
    bool send;
    int peer;
    void* buf;
    int64_t bytes;
  };
  std::vector<DevOp> batch_;
  std::vector<std::function<void()>> batch_then_;  // continuations due after the batch
  // ordering
  std::mutex mu_;
  int64_t next_xid_ = 1;
  std::map<int64_t, std::function<void()>> at_server_;  // xid -> this server's side
  ClientFn at_client_;
  // self-loop: the notice whose server side is being queued; the client side joins the RCCL
  // group of the server's op (a send to self and its receive must be in one ncclGroup)
  bool self_armed_ = false;
  int64_t self_coff_ = 0, self_bytes_ = 0;
  int self_window_ = 0;
  bool self_to_client_ = false;
  void self_join();
  // host FIFO (one per rank: every op of the instance on this rank)
  std::deque<Op> q_;
  std::map<int, int64_t> cts_got_, cts_used_;  // rendezvous: clear-to-send per peer
  int hook_ = -1;
  int jitter_us_ = 0;
  std::mt19937 rng_;
  int64_t bytes_sent_ = 0, bytes_recv_ = 0, ordered_ = 0, groups_ = 0;
};

}  // namespace mpit
