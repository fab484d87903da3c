// One-sided communication windows (MPI_Win_* equivalent, SURVEY §7.1 Tier 2).
//
// A device window is a region of HBM that every member rank maps through HIP IPC, so
// Put / Get are single hipMemcpyAsync peer copies over xGMI and Accumulate is a fused
// HIP kernel that read-modify-writes the remote HBM directly. A host window lives in a
// named POSIX shm object that every member maps. Each rank's window also carries a
// 64-B control block in host shm with a reader/writer lock word (Win_lock/Win_unlock).
//
// The parameter server (ps.h) is built on these windows: every client exposes an "rx"
// window (where pulled parameters land — normally the model's own flat parameter
// memory) and a "tx" window (pushed gradients / parameters), and servers read / write
// them directly, replacing the reference's message copies of whole shards
// (asyncsgd/pclient.lua:49-94, asyncsgd/pserver.lua:65-111).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

#include "engine.h"

namespace mpit {

struct alignas(64) WinCtl {
  std::atomic<int64_t> lock;  // 0 free, >0 shared holders, -1 exclusive
  std::atomic<int64_t> epoch;
  char pad[48];
};

class Window {
 public:
  // local == 0 -> allocate `bytes` (hipMalloc for device windows, shm for host windows)
  Window(Engine& eng, int64_t id, uintptr_t local, int64_t bytes, bool device);
  ~Window();
  Window(const Window&) = delete;
  Window& operator=(const Window&) = delete;

  // this rank's exposure blob (exchange it among the members, then connect())
  std::string blob() const;
  // map_remote=false: leave other ranks' device windows unmapped (PS datapath 3 moves the
  // shard data as messages and never touches a peer allocation)
  void connect(const std::vector<std::string>& blobs, const std::vector<int>& world_ranks, bool map_remote = true);
  void unlink_names();  // after every member connected

  uintptr_t local_ptr() const { return reinterpret_cast<uintptr_t>(local_); }
  int64_t bytes() const { return bytes_; }
  bool device() const { return device_; }
  int members() const { return int(remote_.size()); }
  uintptr_t remote_ptr(int m) const;  // member index
  int64_t remote_bytes(int m) const;
  bool remote_device(int m) const;

  // data movement (member index; offsets in bytes). src/dst device-ness given by caller.
  void put(int m, int64_t off, uintptr_t src, int64_t n, hipStream_t s);
  void get(uintptr_t dst, int m, int64_t off, int64_t n, hipStream_t s);
  // dst[m][off..] = a*src + b*dst (fp32|bf16 elements), atomic w.r.t. other accumulates
  // through the exclusive lock of the target.
  void accumulate(int m, int64_t off, uintptr_t src, bool src_dev, int64_t nelem, bool bf16, float a, float b,
                  hipStream_t s);
  void lock(int m, bool exclusive);
  bool try_lock(int m, bool exclusive);
  void unlock(int m);
  void flush(hipStream_t s);  // complete all operations this rank issued on stream s

 private:
  Engine& eng_;
  int64_t id_;
  int64_t bytes_;
  bool device_;
  bool own_ = false;
  void* local_ = nullptr;
  std::string ctl_name_;
  WinCtl* ctl_ = nullptr;
  void* ctl_map_ = nullptr;
  int64_t ctl_map_bytes_ = 0;
  struct Remote {
    void* ptr = nullptr;
    int64_t bytes = 0;
    bool device = false;
    int world_rank = -1;
    WinCtl* ctl = nullptr;
    void* map = nullptr;
    int64_t map_bytes = 0;
  };
  std::vector<Remote> remote_;
  std::vector<int> held_;  // lock mode held per member: 0 none, 1 shared, 2 exclusive
};

}  // namespace mpit
