// Node-local shared-memory segment: the control plane (and the host data plane) of the
// mpit runtime. Replaces the MPI library underneath mpiT's binding (SURVEY §2.1 N1–N7,
// §2.6 C1–C4) for the single-node, one-process-per-GPU MI355X topology.
//
// Layout (one POSIX shm object per job, created by rank 0, name broadcast at Init):
//   Header | Ring[W][W] | Bulk[W][W] (each + bulk_bytes of payload) | Xchg[W][kXchgBytes]
// Ring[s][d] is a single-producer (rank s) single-consumer (rank d) queue of 128-B
// message headers (tag, context, size, inline payload <= 64 B). Bulk[s][d] is the byte
// stream carrying payloads > 64 B of host messages, in ring order. Xchg is a scratch
// area for small all-gathers (IPC handles of windows, bootstrap data).
// Atomics are lock-free 64-bit, hence address-free and valid across processes.
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>

namespace mpit {

constexpr int kMaxRanks = 64;
constexpr int kRingSlots = 1024;
constexpr int kInline = 64;
constexpr int64_t kXchgBytes = 8192;
constexpr uint64_t kMagic = 0x6d7069745f616d64ull;  // "mpit_amd"

enum MsgKind : int32_t {
  MK_EAGER = 1,  // payload inline in the header
  MK_BULK = 2,   // payload follows in the pair's bulk byte stream
  MK_DEV = 3,    // device payload: receiver pulls it through an IPC mapping (rendezvous)
  MK_ACK = 4,    // completion of a synchronous / rendezvous send (aux0 = sender request id)
  MK_AM = 5,     // active message for a window / PS (handled by the engine, never matched)
};
enum MsgFlags : int32_t { MF_SYNC = 1 };

struct alignas(64) Msg {
  int32_t kind;
  int32_t tag;
  int32_t ctx;
  int32_t src;
  int64_t nbytes;
  int64_t seq;
  int32_t flags;
  int32_t dev;
  int64_t aux0;  // MK_DEV: byte offset inside the exported allocation; MK_ACK: request id
  int64_t aux1;  // MK_DEV / MK_SYNC: sender request id
  int64_t aux2;
  uint8_t data[kInline];
};
static_assert(sizeof(Msg) == 128, "Msg must be 128 bytes");

struct alignas(64) Ring {
  std::atomic<uint64_t> head;  // next slot the producer writes
  char pad0[56];
  std::atomic<uint64_t> tail;  // next slot the consumer reads
  char pad1[56];
  Msg slots[kRingSlots];
};

struct alignas(64) BulkHdr {
  std::atomic<uint64_t> wpos;
  char pad0[56];
  std::atomic<uint64_t> rpos;
  char pad1[56];
};

struct alignas(64) RankInfo {
  std::atomic<int32_t> attached;
  int32_t pid;
  int32_t device;
  int32_t pad;
  char host[48];
  // An idle progress thread parks on `doorbell` (a futex word shared across processes)
  // after announcing itself in `sleeping`; whoever hands it work (a ring message, bulk
  // bytes, a freed ring slot, a local request) bumps the word and wakes it (engine.cpp).
  alignas(64) std::atomic<uint32_t> doorbell;
  std::atomic<int32_t> sleeping;
};

constexpr int kAbortMsg = 256;

struct alignas(64) Header {
  uint64_t magic;
  int32_t world;
  int32_t ring_slots;
  int64_t bulk_bytes;
  int64_t total_bytes;
  std::atomic<int32_t> nattached;
  std::atomic<int32_t> abort_flag;
  int32_t abort_code;
  int32_t abort_rank;  // the rank that raised the fatal error (abort_msg is its reason)
  char abort_msg[kAbortMsg];
  alignas(64) std::atomic<uint64_t> bar_count;
  alignas(64) std::atomic<uint64_t> bar_gen;
  alignas(64) RankInfo ranks[kMaxRanks];
};

class Segment {
 public:
  // rank 0 creates (create=true), others attach. world <= kMaxRanks.
  Segment(const std::string& name, int world, int rank, bool create, int64_t bulk_bytes);
  ~Segment();
  Segment(const Segment&) = delete;
  Segment& operator=(const Segment&) = delete;

  Header* hdr() const { return hdr_; }
  Ring* ring(int src, int dst) const;
  BulkHdr* bulk(int src, int dst) const;
  uint8_t* bulk_data(int src, int dst) const { return reinterpret_cast<uint8_t*>(bulk(src, dst)) + sizeof(BulkHdr); }
  uint8_t* xchg(int r) const { return xchg_ + r * kXchgBytes; }
  int64_t bulk_bytes() const { return bulk_bytes_; }
  int world() const { return world_; }
  void unlink();  // remove the name (mapping stays valid) — done once all ranks attached
  const std::string& name() const { return name_; }

  static int64_t layout_bytes(int world, int64_t bulk_bytes);

 private:
  std::string name_;
  int world_;
  int64_t bulk_bytes_;
  int64_t size_ = 0;
  void* base_ = nullptr;
  Header* hdr_ = nullptr;
  uint8_t* rings_ = nullptr;
  uint8_t* bulks_ = nullptr;
  uint8_t* xchg_ = nullptr;
  bool unlinked_ = false;
};

}  // namespace mpit
