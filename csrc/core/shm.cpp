#include "shm.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <new>
#include <stdexcept>
#include <thread>

namespace mpit {

namespace {
int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }
}  // namespace

int64_t Segment::layout_bytes(int world, int64_t bulk_bytes) {
  int64_t s = align_up(sizeof(Header), 4096);
  s += align_up(int64_t(sizeof(Ring)) * world * world, 4096);
  s += align_up((int64_t(sizeof(BulkHdr)) + bulk_bytes) * world * world, 4096);
  s += align_up(kXchgBytes * world, 4096);
  return s;
}

Segment::Segment(const std::string& name, int world, int rank, bool create, int64_t bulk_bytes)
    : name_(name), world_(world), bulk_bytes_(align_up(bulk_bytes, 4096)) {
  if (world < 1 || world > kMaxRanks) throw std::invalid_argument("mpit: world size out of range (1..64)");
  size_ = layout_bytes(world, bulk_bytes_);
  int fd = -1;
  if (create) {
    ::shm_unlink(name.c_str());
    fd = ::shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("mpit: shm_open(create) failed for " + name + ": " + strerror(errno));
    if (::ftruncate(fd, size_) != 0) {
      ::close(fd);
      throw std::runtime_error("mpit: ftruncate failed: " + std::string(strerror(errno)));
    }
  } else {
    auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      fd = ::shm_open(name.c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (::fstat(fd, &st) == 0 && st.st_size >= size_) break;
        ::close(fd);
        fd = -1;
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
        throw std::runtime_error("mpit: timed out attaching shm segment " + name);
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
  }
  base_ = ::mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (base_ == MAP_FAILED) throw std::runtime_error("mpit: mmap of shm segment failed");
  uint8_t* b = static_cast<uint8_t*>(base_);
  hdr_ = reinterpret_cast<Header*>(b);
  rings_ = b + align_up(sizeof(Header), 4096);
  bulks_ = rings_ + align_up(int64_t(sizeof(Ring)) * world * world, 4096);
  xchg_ = bulks_ + align_up((int64_t(sizeof(BulkHdr)) + bulk_bytes_) * world * world, 4096);
  if (create) {
    // ftruncate zero-fills; placement-initialise the atomics explicitly anyway.
    new (&hdr_->nattached) std::atomic<int32_t>(0);
    new (&hdr_->abort_flag) std::atomic<int32_t>(0);
    new (&hdr_->bar_count) std::atomic<uint64_t>(0);
    new (&hdr_->bar_gen) std::atomic<uint64_t>(0);
    hdr_->abort_rank = -1;
    for (int r = 0; r < kMaxRanks; ++r) {
      new (&hdr_->ranks[r].doorbell) std::atomic<uint32_t>(0);
      new (&hdr_->ranks[r].sleeping) std::atomic<int32_t>(0);
    }
    for (int s = 0; s < world; ++s)
      for (int d = 0; d < world; ++d) {
        new (&ring(s, d)->head) std::atomic<uint64_t>(0);
        new (&ring(s, d)->tail) std::atomic<uint64_t>(0);
        new (&bulk(s, d)->wpos) std::atomic<uint64_t>(0);
        new (&bulk(s, d)->rpos) std::atomic<uint64_t>(0);
      }
    hdr_->world = world;
    hdr_->ring_slots = kRingSlots;
    hdr_->bulk_bytes = bulk_bytes_;
    hdr_->total_bytes = size_;
    std::atomic_thread_fence(std::memory_order_release);
    reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->store(kMagic, std::memory_order_release);
  } else {
    auto t0 = std::chrono::steady_clock::now();
    while (reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->load(std::memory_order_acquire) != kMagic) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
        throw std::runtime_error("mpit: shm segment never initialised by rank 0");
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (hdr_->world != world) throw std::runtime_error("mpit: shm segment world size mismatch");
  }
  (void)rank;
}

Segment::~Segment() {
  if (base_ && base_ != MAP_FAILED) ::munmap(base_, size_);
}

void Segment::unlink() {
  if (!unlinked_) {
    ::shm_unlink(name_.c_str());
    unlinked_ = true;
  }
}

Ring* Segment::ring(int src, int dst) const {
  return reinterpret_cast<Ring*>(rings_ + int64_t(sizeof(Ring)) * (int64_t(src) * world_ + dst));
}

BulkHdr* Segment::bulk(int src, int dst) const {
  return reinterpret_cast<BulkHdr*>(bulks_ + (int64_t(sizeof(BulkHdr)) + bulk_bytes_) * (int64_t(src) * world_ + dst));
}

}  // namespace mpit
