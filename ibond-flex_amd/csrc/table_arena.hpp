// Device memory for the fixed-base tables (flexpai.hip ensure_fb / ensure_pfb): tens to hundreds of GB per context,
// built once per key and window. They come from a process-wide pool of physical chunks that are mapped into a fresh
// virtual range per table (HIP virtual memory management: hipMemCreate, hipMemAddressReserve, hipMemMap), and a
// released table returns its chunks to the pool instead of to the driver. Reason (round 6, tools/pfb_setup_trace.py,
// profiles/r06c_pfb_setup_trace.log): the driver wipes released VRAM before it hands it out again, so the 139 GB public
// tables took 2.5 s to ALLOCATE after a key holder's 177 GB were released, 5.9 s after a second rebuild, and 0.9 ms on
// untouched memory. A process that rebuilds tables -- a new window, a re-keyed exchange (HE_SA_FT), the public leg after
// the key holder's -- reuses memory it already owns. Chunks go back to the driver when the process's last context is
// destroyed (pai_ctx_destroy) or on pai_release_table_cache(). $FLEXPAI_TABLE_POOL=0, or a runtime without virtual
// memory management, allocates the tables with hipMalloc / hipFree.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

namespace fpai {

class TableArena {
 public:
  static TableArena& get() {
    static TableArena a;
    return a;
  }

  // device memory for `bytes` on the current device (hipSetDevice done by the caller), or nullptr
  void* alloc(int device, size_t bytes) {
    if (!enabled()) return plain_alloc(bytes);
    std::lock_guard<std::mutex> lk(mu_);
    const size_t cb = chunk_bytes(device);
    if (!cb) return plain_alloc_locked(bytes);
    const size_t nch = (bytes + cb - 1) / cb;
    void* va = nullptr;
    if (hipMemAddressReserve(&va, nch * cb, cb, nullptr, 0) != hipSuccess) {
      (void)hipGetLastError();
      return plain_alloc_locked(bytes);
    }
    Map m{device, nch * cb, {}};
    std::vector<hipMemGenericAllocationHandle_t>& pool = pool_[device];
    for (size_t i = 0; i < nch; ++i) {
      hipMemGenericAllocationHandle_t h{};
      if (!pool.empty()) {
        h = pool.back();
        pool.pop_back();
      } else {
        hipMemAllocationProp prop = props(device);
        if (hipMemCreate(&h, cb, &prop, 0) != hipSuccess) {
          (void)hipGetLastError();
          unwind(va, m);
          return nullptr;
        }
      }
      if (hipMemMap((char*)va + i * cb, cb, 0, h, 0) != hipSuccess) {
        (void)hipGetLastError();
        pool.push_back(h);
        unwind(va, m);
        return nullptr;
      }
      m.chunks.push_back(h);
    }
    hipMemAccessDesc acc{};
    acc.location.type = hipMemLocationTypeDevice;
    acc.location.id = device;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    if (hipMemSetAccess(va, nch * cb, &acc, 1) != hipSuccess) {
      (void)hipGetLastError();
      unwind(va, m);
      return nullptr;
    }
    maps_[va] = std::move(m);
    return va;
  }

  void free(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(mu_);
    auto it = maps_.find(p);
    if (it == maps_.end()) {
      (void)hipFree(p);
      return;
    }
    (void)hipDeviceSynchronize();   // (the table's last readers; frees are rare: a rebuild or a context's end)
    unwind(p, it->second);
    maps_.erase(it);
  }

  // chunks held for reuse on `device` (fb_budget counts them as free)
  size_t pooled_bytes(int device) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = pool_.find(device);
    return it == pool_.end() ? 0 : it->second.size() * chunk_bytes(device);
  }

  bool pooled_any() {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& kv : pool_)
      if (!kv.second.empty()) return true;
    return false;
  }

  // every pooled chunk back to the driver
  void trim() {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& kv : pool_) {
      for (hipMemGenericAllocationHandle_t h : kv.second) (void)hipMemRelease(h);
      kv.second.clear();
    }
  }

 private:
  struct Map {
    int device = 0;
    size_t bytes = 0;
    std::vector<hipMemGenericAllocationHandle_t> chunks;
  };
  std::mutex mu_;
  std::map<int, std::vector<hipMemGenericAllocationHandle_t>> pool_;
  std::map<void*, Map> maps_;
  std::map<int, size_t> chunk_;

  static bool enabled() {
    static const bool on = [] {
      const char* e = getenv("FLEXPAI_TABLE_POOL");
      return !e || atoi(e) != 0;
    }();
    return on;
  }
  static hipMemAllocationProp props(int device) {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    return prop;
  }
  // 1 GiB chunks (a multiple of the allocation granularity): a table wastes less than one chunk
  size_t chunk_bytes(int device) {
    auto it = chunk_.find(device);
    if (it != chunk_.end()) return it->second;
    size_t g = 0;
    hipMemAllocationProp prop = props(device);
    size_t cb = 0;
    if (hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended) == hipSuccess && g) {
      cb = ((size_t(1) << 30) + g - 1) / g * g;
    } else {
      (void)hipGetLastError();
    }
    chunk_[device] = cb;
    return cb;
  }
  static void* plain_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    return p;
  }
  void* plain_alloc_locked(size_t bytes) { return plain_alloc(bytes); }
  // unmap what `m` mapped at va, return its chunks to the pool, release the range
  void unwind(void* va, Map& m) {
    const size_t cb = chunk_bytes(m.device);
    for (size_t i = 0; i < m.chunks.size(); ++i) {
      (void)hipMemUnmap((char*)va + i * cb, cb);
      pool_[m.device].push_back(m.chunks[i]);
    }
    m.chunks.clear();
    (void)hipMemAddressFree(va, m.bytes);
    (void)hipGetLastError();
  }
};

}  // namespace fpai
