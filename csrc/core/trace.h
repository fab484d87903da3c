// roctx ranges from the native runtime (the server's progress thread: shard updates, pulls,
// parameter pushes), so rocprofv3 --marker-trace shows the parameter server next to the
// Python-side ranges of mpit_amd/utils/trace.py. The roctx library is opened at run time and
// only when MPIT_TRACE=1: no link dependency, nothing done otherwise. rocprofv3 intercepts
// the rocprofiler-sdk roctx library (ROCm 7); the legacy libroctx64 is the fallback.
#pragma once
#include <dlfcn.h>

#include <cstdlib>
#include <cstring>

namespace mpit {

struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  static const Roctx& get() {
    static const Roctx r = [] {
      Roctx x;
      const char* e = std::getenv("MPIT_TRACE");
      if (!e || std::strcmp(e, "1") != 0) return x;
      void* h = nullptr;
      for (const char* n : {"librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                            "libroctx64.so", "/opt/rocm/lib/libroctx64.so"})
        if (!h) h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
      if (!h) return x;
      x.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      x.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
      if (!x.push || !x.pop) x.push = nullptr;
      return x;
    }();
    return r;
  }
};

// scoped range; a no-op unless tracing is on
class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(Roctx::get().push != nullptr) {
    if (on_) Roctx::get().push(name);
  }
  ~TraceRange() {
    if (on_) Roctx::get().pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

}  // namespace mpit
