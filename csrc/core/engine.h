// mpit native runtime engine: tagged, probe-able, cancellable non-blocking point-to-point
// messaging between the ranks of one node, a progress thread, world barrier, small
// all-gather, and device-buffer rendezvous over HIP IPC (xGMI peer copies).
//
// What it replaces in the reference:
//   N1–N7  C/MPI binding  -> this engine + mpit_amd/comm.py (hand-written API subset)
//   R2/R3  aio_send/aio_recv (coroutines polling Isend/Iprobe/Irecv/Test, init.lua:41-108)
//          -> Engine::isend/irecv + a C++ progress thread; Python waits with the GIL
//             released instead of resuming coroutines (init.lua:139-192).
//   C3     tagged control plane (asyncsgd/init.lua:3-10), C6 cancellation (init.lua:53-59)
//          -> MPI matching on (context, source, tag) with ANY_SOURCE/ANY_TAG, Iprobe,
//             Cancel for unmatched receives as well as unstarted sends (the reference's
//             receive-cancel branch is unreachable, init.lua:94-102 — fixed here).
//   C8     GPU-direct through CUDA-aware MPI (lua-mpi.h:78) -> MK_DEV rendezvous: the
//          receiver pulls the sender's HBM buffer with hipMemcpyAsync over xGMI.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "shm.h"

namespace mpit {

constexpr int kAnySource = -1;
constexpr int kAnyTag = -1;

// Raw futex on a 32-bit word. shared: the word lives in the cross-process segment.
// futex_wait returns when woken, when *addr != expect, or after timeout_us (< 0: none).
void futex_wake_all(void* addr, bool shared);
void futex_wait(void* addr, uint32_t expect, int64_t timeout_us, bool shared);

struct Status {
  int source = -1;
  int tag = -1;
  int error = 0;
  int64_t count = 0;  // bytes
  bool cancelled = false;
};

enum ReqState : int { RS_PENDING = 0, RS_DONE = 1, RS_CANCELLED = 2, RS_ERROR = 3 };

struct Req {
  int64_t id = 0;
  bool is_send = false;
  std::atomic<int> state{RS_PENDING};
  Status st;
  std::string err;
  // send
  int dst = -1;
  const uint8_t* sbuf = nullptr;
  int64_t nbytes = 0;
  bool sdev = false;
  int sdevice = -1;
  bool sync = false;
  bool header_posted = false;
  int64_t sent = 0;
  // recv
  int src = kAnySource;
  uint8_t* rbuf = nullptr;
  int64_t cap = 0;
  bool rdev = false;
  int rdevice = -1;
  int tag = 0;
  int ctx = 0;
};

// One in-progress message, either matched to a receive or parked as unexpected.
struct Incoming {
  Msg hdr;
  std::vector<uint8_t> data;  // heap copy (unexpected, or staging for a device receive)
  int64_t got = 0;            // payload bytes received so far (bulk)
  bool complete = false;
  std::shared_ptr<Req> req;   // set once matched
};

struct PendingCopy {  // an outstanding hipMemcpyAsync whose completion finishes a request
  hipEvent_t ev;
  std::shared_ptr<Req> req;
  int ack_to = -1;      // rank to send MK_ACK to on completion (rendezvous)
  int64_t ack_id = 0;
  std::function<void()> then;  // optional continuation (runs on the progress thread)
  int ipc_owner = -1;          // an IPC mapping the copy reads (released on completion)
  std::string ipc_key;
};

struct IpcMapping {  // an opened peer allocation (receiver side)
  void* ptr = nullptr;
  uint64_t last_use = 0;
  int64_t inflight = 0;  // copies reading it; permanent (window) mappings hold kPinned
};

class Engine {
 public:
  Engine(const std::string& shm_name, int world, int rank, bool create, int device, int64_t bulk_bytes);
  ~Engine();

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  Segment& seg() { return *seg_; }

  // point-to-point (nbytes in bytes; device buffers flagged with dev=true)
  int64_t isend(const void* buf, int64_t nbytes, bool dev, int dst, int tag, int ctx, bool sync);
  int64_t irecv(void* buf, int64_t cap, bool dev, int src, int tag, int ctx);
  // returns true when complete (status filled); frees the request unless keep
  bool test(int64_t id, Status* st, bool keep = false);
  void wait(int64_t id, Status* st);
  bool cancel(int64_t id);
  void free_request(int64_t id);
  bool iprobe(int src, int tag, int ctx, Status* st);
  void probe(int src, int tag, int ctx, Status* st);

  // world-level collectives through the shm segment
  void barrier();
  std::vector<std::string> allgather_small(const std::string& blob);

  // active messages (control-only, payload <= 64 B), handled on the progress thread
  using AmHandler = std::function<void(const Msg&)>;
  void register_am(int id, AmHandler h);
  void send_am(int dst, int id, const void* payload, int64_t n, int64_t aux0 = 0, int64_t aux1 = 0,
               int64_t aux2 = 0);
  // periodic hooks run by the progress thread each iteration (PS server state machines)
  int add_hook(std::function<bool()> h);
  void remove_hook(int id);
  // track an async device copy; `then` runs on the progress thread when it is done
  void track_copy(hipEvent_t ev, std::function<void()> then);
  // pooled completion events (no hipEventCreate / Destroy per message): events handed to
  // track_copy return to the pool when their copy is done
  hipEvent_t get_event();
  void put_event(hipEvent_t e);
  static void record_event(hipEvent_t e, hipStream_t s);

  void abort(int code);
  // A fatal error of this rank's runtime (a failed active-message handler, a failed HIP
  // call on the progress thread): publish the reason in the segment, raise the job-wide
  // abort flag, wake every rank and exit. Every other rank then prints the reason and
  // exits with the same code — the reference's co_ping assert(false), init.lua:168-171.
  [[noreturn]] void fatal(const std::string& why, int code = 71);
  void shutdown();

  // wake rank r's progress thread if it is parked on its doorbell
  void ring(int r);
  // new local work for this rank's progress thread (a posted request, a gated send)
  void kick();
  // outstanding GPU-side completions polled by hooks (PS gates): while > 0 the progress
  // thread polls every ~20 us instead of parking on its doorbell
  void gpu_pending_add(int64_t d) {
    gpu_pending_.fetch_add(d, std::memory_order_acq_rel);
    if (d > 0) kick();
  }
  // deadlines (seconds, 0 = none): MPIT_WAIT_TIMEOUT_S for Wait/Probe/Barrier
  static double wait_timeout_s();

  hipStream_t comm_stream() const { return stream_; }
  // IPC helpers (also used by windows)
  static void export_ptr(const void* p, hipIpcMemHandle_t* h, int64_t* offset, int64_t* alloc_bytes);
  // export with a per-allocation handle cache (keyed by the allocation's unique buffer id,
  // so a recycled address range never reuses a stale handle)
  void export_cached(const void* p, hipIpcMemHandle_t* h, int64_t* offset);
  // open (or reuse) a peer allocation. permanent: a window mapping, never evicted;
  // otherwise the caller holds it for one copy and returns it with release_ipc
  void* open_ipc(int owner_rank, const hipIpcMemHandle_t& h, bool permanent = true);
  void release_ipc(int owner_rank, const std::string& key);

  // statistics
  int64_t bytes_sent() const { return bytes_sent_.load(); }
  int64_t bytes_recv() const { return bytes_recv_.load(); }
  int64_t msgs_sent() const { return msgs_sent_.load(); }

 private:
  void progress_loop();
  void check_peers();
  bool progress_once();
  bool progress_sends_locked();
  bool progress_recvs_locked();
  bool progress_copies();
  void check_abort();
  void publish_abort(const std::string& why, int code);
  bool idle_deep_ok();
  void park(int64_t timeout_us, uint64_t last_act);
  bool push_msg_locked(int dst, const Msg& m);
  int64_t bulk_write_locked(int dst, const uint8_t* p, int64_t n);
  int64_t bulk_read(int src, uint8_t* p, int64_t n);
  bool match(const Msg& h, const Req& r) const;
  void on_header_locked(int src, const Msg& h);
  void deliver_locked(Incoming& in);
  void start_dev_pull_locked(Incoming& in);
  void finish_req(const std::shared_ptr<Req>& r, int state);
  std::shared_ptr<Req> get_req(int64_t id);

  std::unique_ptr<Segment> seg_;
  int world_, rank_, device_;
  hipStream_t stream_ = nullptr;

  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<bool> running_{true};
  std::thread thread_;

  std::atomic<int64_t> next_id_{1};
  std::unordered_map<int64_t, std::shared_ptr<Req>> reqs_;
  std::vector<std::deque<std::shared_ptr<Req>>> sendq_;          // per destination, FIFO
  std::vector<std::deque<Msg>> ctrlq_;                            // per destination control msgs
  std::list<std::shared_ptr<Req>> posted_;                        // posted receives, post order
  std::list<std::shared_ptr<Incoming>> unexpected_;               // arrival order
  std::vector<std::shared_ptr<Incoming>> streaming_;              // per source: bulk in progress
  std::map<int64_t, std::shared_ptr<Req>> await_ack_;             // sync / rendezvous sends
  std::vector<int64_t> send_seq_;

  std::mutex copy_mu_;
  std::vector<PendingCopy> copies_;
  std::mutex ev_mu_;
  std::vector<hipEvent_t> ev_pool_;

  std::mutex am_mu_;
  std::unordered_map<int, AmHandler> am_;
  std::vector<Msg> pending_am_;
  std::list<Msg> orphan_am_;  // arrived before their handler was registered
  std::mutex hook_mu_;
  std::map<int, std::function<bool()>> hooks_;
  int next_hook_ = 1;

  std::mutex ipc_mu_;
  std::map<std::pair<int, std::string>, IpcMapping> ipc_cache_;
  uint64_t ipc_tick_ = 0;
  // LRU bound on transient peer mappings: a mapping keeps the exporter's (possibly freed
  // and recycled) allocation alive, so idle ones are closed once the cache is full
  static constexpr size_t kIpcCacheMax = 256;
  static constexpr int64_t kPinned = int64_t(1) << 40;
  std::mutex export_mu_;
  std::unordered_map<uint64_t, std::pair<hipIpcMemHandle_t, uintptr_t>> export_cache_;  // buffer id -> (handle, base)

  std::atomic<int64_t> bytes_sent_{0}, bytes_recv_{0}, msgs_sent_{0};
  std::atomic<uint64_t> activity_{0};
  std::atomic<int64_t> gpu_pending_{0};
  uint64_t bar_local_gen_ = 0;
};

}  // namespace mpit
