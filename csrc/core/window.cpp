#include "window.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <xmmintrin.h>

#include <chrono>
#include <cstring>
#include <new>
#include <stdexcept>
#include <thread>

#include "../kernels/kernels.h"

namespace mpit {

namespace {

void hipw(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("mpit window HIP error in ") + what + ": " + hipGetErrorString(e));
}

struct Blob {
  int64_t bytes;
  int32_t device;
  int32_t world_rank;
  int64_t offset;
  hipIpcMemHandle_t handle;
  char ctl_name[160];
};

void* map_named(const std::string& name, int64_t bytes, bool create) {
  int fd;
  if (create) {
    ::shm_unlink(name.c_str());
    fd = ::shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("mpit: window shm_open(create) failed: " + name);
    if (::ftruncate(fd, bytes) != 0) {
      ::close(fd);
      throw std::runtime_error("mpit: window ftruncate failed");
    }
  } else {
    fd = ::shm_open(name.c_str(), O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("mpit: window shm_open(attach) failed: " + name);
  }
  void* p = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("mpit: window mmap failed");
  return p;
}

constexpr int64_t kCtl = 64;

}  // namespace

Window::Window(Engine& eng, int64_t id, uintptr_t local, int64_t bytes, bool device)
    : eng_(eng), id_(id), bytes_(bytes), device_(device) {
  if (device && eng.device() < 0) throw std::invalid_argument("mpit: device window on a rank without a device");
  ctl_name_ = eng.seg().name() + "_w" + std::to_string(id) + "_r" + std::to_string(eng.rank());
  ctl_map_bytes_ = kCtl + (device ? 0 : std::max<int64_t>(bytes, 0));
  ctl_map_ = map_named(ctl_name_, std::max<int64_t>(ctl_map_bytes_, 64), true);
  ctl_ = new (ctl_map_) WinCtl();
  ctl_->lock.store(0);
  ctl_->epoch.store(0);
  if (device) {
    if (local) {
      local_ = reinterpret_cast<void*>(local);
    } else if (bytes > 0) {
      hipw(hipSetDevice(eng.device()), "hipSetDevice");
      hipw(hipMalloc(&local_, size_t(bytes)), "hipMalloc(window)");
      hipw(hipMemset(local_, 0, size_t(bytes)), "hipMemset(window)");
      own_ = true;
    }
  } else {
    local_ = static_cast<uint8_t*>(ctl_map_) + kCtl;
    if (local && bytes > 0) std::memcpy(local_, reinterpret_cast<const void*>(local), size_t(bytes));
  }
}

Window::~Window() {
  for (auto& r : remote_)
    if (r.map && r.map != ctl_map_) ::munmap(r.map, std::max<int64_t>(r.map_bytes, 64));
  if (ctl_map_) ::munmap(ctl_map_, std::max<int64_t>(ctl_map_bytes_, 64));
  ::shm_unlink(ctl_name_.c_str());
  if (own_ && local_) {
    hipSetDevice(eng_.device());
    hipFree(local_);
  }
}

std::string Window::blob() const {
  Blob b{};
  b.bytes = bytes_;
  b.device = device_ ? 1 : 0;
  b.world_rank = eng_.rank();
  std::strncpy(b.ctl_name, ctl_name_.c_str(), sizeof(b.ctl_name) - 1);
  if (device_ && local_ && bytes_ > 0) {
    hipw(hipSetDevice(eng_.device()), "hipSetDevice");
    Engine::export_ptr(local_, &b.handle, &b.offset, nullptr);
  }
  return std::string(reinterpret_cast<const char*>(&b), sizeof(b));
}

void Window::connect(const std::vector<std::string>& blobs, const std::vector<int>& world_ranks, bool map_remote) {
  remote_.assign(blobs.size(), Remote{});
  held_.assign(blobs.size(), 0);
  for (size_t m = 0; m < blobs.size(); ++m) {
    if (blobs[m].size() != sizeof(Blob)) throw std::invalid_argument("mpit: bad window blob");
    Blob b;
    std::memcpy(&b, blobs[m].data(), sizeof(b));
    Remote& r = remote_[m];
    r.bytes = b.bytes;
    r.device = b.device != 0;
    r.world_rank = b.world_rank;
    if (world_ranks.size() == blobs.size() && world_ranks[m] != b.world_rank)
      throw std::invalid_argument("mpit: window member order mismatch");
    if (b.world_rank == eng_.rank()) {
      r.ptr = local_;
      r.ctl = ctl_;
      r.map = ctl_map_;
      continue;
    }
    r.map_bytes = kCtl + (r.device ? 0 : std::max<int64_t>(b.bytes, 0));
    r.map = map_named(b.ctl_name, std::max<int64_t>(r.map_bytes, 64), false);
    r.ctl = static_cast<WinCtl*>(r.map);
    if (!r.device) {
      r.ptr = static_cast<uint8_t*>(r.map) + kCtl;
    } else if (b.bytes > 0 && eng_.device() >= 0 && map_remote) {
      try {
        r.ptr = static_cast<uint8_t*>(eng_.open_ipc(b.world_rank, b.handle)) + b.offset;
      } catch (const std::exception& e) {
        // name the pair: which rank (device) could not map whose window (device)
        throw std::runtime_error("mpit: rank " + std::to_string(eng_.rank()) + " (device " +
                                 std::to_string(eng_.device()) + ") could not map window " + std::to_string(id_) +
                                 " of rank " + std::to_string(b.world_rank) + ": " + e.what());
      }
    }
  }
}

void Window::unlink_names() { ::shm_unlink(ctl_name_.c_str()); }

uintptr_t Window::remote_ptr(int m) const { return reinterpret_cast<uintptr_t>(remote_.at(size_t(m)).ptr); }
int64_t Window::remote_bytes(int m) const { return remote_.at(size_t(m)).bytes; }
bool Window::remote_device(int m) const { return remote_.at(size_t(m)).device; }

void Window::put(int m, int64_t off, uintptr_t src, int64_t n, hipStream_t s) {
  const Remote& r = remote_.at(size_t(m));
  if (off < 0 || off + n > r.bytes) throw std::out_of_range("mpit: Put outside the target window");
  if (!r.ptr && n > 0) throw std::runtime_error("mpit: target window not mapped on this rank");
  uint8_t* dst = static_cast<uint8_t*>(r.ptr) + off;
  if (eng_.device() >= 0) {
    hipw(hipSetDevice(eng_.device()), "hipSetDevice");
    hipw(hipMemcpyAsync(dst, reinterpret_cast<const void*>(src), size_t(n), hipMemcpyDefault, s), "Put");
  } else {
    std::memcpy(dst, reinterpret_cast<const void*>(src), size_t(n));
  }
}

void Window::get(uintptr_t dst, int m, int64_t off, int64_t n, hipStream_t s) {
  const Remote& r = remote_.at(size_t(m));
  if (off < 0 || off + n > r.bytes) throw std::out_of_range("mpit: Get outside the target window");
  if (!r.ptr && n > 0) throw std::runtime_error("mpit: target window not mapped on this rank");
  const uint8_t* src = static_cast<const uint8_t*>(r.ptr) + off;
  if (eng_.device() >= 0) {
    hipw(hipSetDevice(eng_.device()), "hipSetDevice");
    hipw(hipMemcpyAsync(reinterpret_cast<void*>(dst), src, size_t(n), hipMemcpyDefault, s), "Get");
  } else {
    std::memcpy(reinterpret_cast<void*>(dst), src, size_t(n));
  }
}

void Window::accumulate(int m, int64_t off, uintptr_t src, bool src_dev, int64_t nelem, bool bf16, float a, float b,
                        hipStream_t s) {
  const Remote& r = remote_.at(size_t(m));
  const int64_t es = bf16 ? 2 : 4;
  if (off < 0 || off + nelem * es > r.bytes) throw std::out_of_range("mpit: Accumulate outside the target window");
  uint8_t* dst = static_cast<uint8_t*>(r.ptr) + off;
  lock(m, true);
  try {
    const uint32_t bf = bf16 ? 3u : 0u;
    if (r.device) {
      if (!src_dev) throw std::invalid_argument("mpit: Accumulate into a device window needs a device origin buffer");
      ew_update(kAxpby, 0, eng_.device(), s, nelem, {reinterpret_cast<uintptr_t>(dst), src}, bf, {a, b});
      hipw(hipStreamSynchronize(s), "Accumulate sync");
    } else {
      if (src_dev) throw std::invalid_argument("mpit: Accumulate into a host window needs a host origin buffer");
      ew_update(kAxpby, 0, -1, nullptr, nelem, {reinterpret_cast<uintptr_t>(dst), src}, bf, {a, b});
    }
  } catch (...) {
    unlock(m);
    throw;
  }
  unlock(m);
}

bool Window::try_lock(int m, bool exclusive) {
  WinCtl* c = remote_.at(size_t(m)).ctl;
  int64_t v = c->lock.load(std::memory_order_acquire);
  if (exclusive) {
    int64_t z = 0;
    if (c->lock.compare_exchange_strong(z, -1, std::memory_order_acq_rel)) {
      held_[size_t(m)] = 2;
      return true;
    }
    return false;
  }
  if (v < 0) return false;
  if (c->lock.compare_exchange_strong(v, v + 1, std::memory_order_acq_rel)) {
    held_[size_t(m)] = 1;
    return true;
  }
  return false;
}

void Window::lock(int m, bool exclusive) {
  int spins = 0;
  while (!try_lock(m, exclusive)) {
    if (++spins < 1000) _mm_pause();
    else std::this_thread::sleep_for(std::chrono::microseconds(5));
  }
}

void Window::unlock(int m) {
  WinCtl* c = remote_.at(size_t(m)).ctl;
  const int h = held_.at(size_t(m));
  if (h == 2) c->lock.store(0, std::memory_order_release);
  else if (h == 1) c->lock.fetch_sub(1, std::memory_order_acq_rel);
  else throw std::runtime_error("mpit: Win_unlock without a matching Win_lock");
  held_[size_t(m)] = 0;
}

void Window::flush(hipStream_t s) {
  if (eng_.device() >= 0) {
    hipw(hipSetDevice(eng_.device()), "hipSetDevice");
    hipw(hipStreamSynchronize(s), "Win_flush");
  }
}

}  // namespace mpit
