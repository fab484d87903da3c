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
// Ordering (deadlock freedom): one 2-rank RCCL communicator per (client, server) pair of
// distinct ranks, server = communicator rank 0. A pair's communicator carries only that
// pair's PS data, in control-plane order: the client posts send(grad) [recv(param)] /
// recv(param) / send(param) in its call order right after the matching control message, the
// server posts recv(grad) [send(param)] / send(param) / recv(param) in the order the pair's
// control messages arrive (one FIFO ring per rank pair), so the two op sequences of every
// communicator are identical. A worker's client ops run on its own client stream and a
// server's on its link streams, so no stream ever holds a client op behind a server op of
// the same rank. A deferred (SSP) pull is sent late, but its client cannot post the next
// push before that pull has arrived (it waits for it), so nothing is queued behind it.
// Every RCCL call of a rank is made by its progress thread (one thread per communicator).
//
// Without a GPU (the CPU test tier) the same op sequence runs over the engine's tagged host
// messages (Engine::isend / irecv, FIFO per (source, tag, context)), the engine standing in
// for RCCL: tests/mp/ps_link.py checks the ordering there, co-located and 1 + k dedicated.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "engine.h"

namespace mpit {

class PsLink {
 public:
  // servers / clients: world ranks of the PS instance's roles; device: RCCL between GPUs,
  // else the engine's host messages
  PsLink(Engine& eng, int ps_id, std::vector<int> servers, std::vector<int> clients, bool device);
  ~PsLink();
  PsLink(const PsLink&) = delete;
  PsLink& operator=(const PsLink&) = delete;

  bool device() const { return device_; }
  // RCCL: a fresh unique id for every pair this rank serves: (client rank, 128-byte id). The
  // caller all-gathers them over the PS group and hands the union to connect() on every
  // member (host transport: empty).
  std::vector<std::pair<int, std::string>> make_ids();
  // (server, client, id) of every pair of the instance; this rank initialises the
  // communicators of its own pairs in one RCCL group (collective over the pairs' ranks)
  void connect(const std::vector<std::tuple<int, int, std::string>>& ids);

  // Queue a transfer with `peer`; as_server names this rank's role in the pair. Device:
  // stream-ordered on s. Host: asynchronous, completing in post order per (peer, role).
  void send(int peer, bool as_server, const void* buf, int64_t bytes, hipStream_t s);
  void recv(int peer, bool as_server, void* buf, int64_t bytes, hipStream_t s);
  // f runs on the progress thread once everything queued so far on s (device) / with
  // (peer, role) (host) has completed
  void then(int peer, bool as_server, hipStream_t s, std::function<void()> f);

  int64_t bytes_sent() const { return bytes_sent_; }
  int64_t bytes_recv() const { return bytes_recv_; }

 private:
  struct Item {
    int64_t req = -1;          // engine request (host), or -1 for a continuation
    std::function<void()> f;   // continuation
  };
  bool poll();  // host: retire completed requests / run due continuations (engine hook)
  void* comm_of(int peer, bool as_server) const;
  int tag_of(bool from_server) const { return from_server ? 2 : 1; }

  Engine& eng_;
  int ps_id_;
  std::vector<int> servers_, clients_;
  bool device_;
  int ctx_;
  // RCCL communicators keyed by (server, client)
  std::map<std::pair<int, int>, void*> comms_;
  // host: per (peer, role) FIFO of outstanding requests and continuations
  std::mutex mu_;
  std::map<std::pair<int, bool>, std::deque<Item>> q_;
  int hook_ = -1;
  int64_t bytes_sent_ = 0, bytes_recv_ = 0;
};

}  // namespace mpit
