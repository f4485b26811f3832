// Pinned-host and HBM buffer pools (see va_allocator.h).
#include "va_allocator.h"

#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <unordered_map>

namespace vision {
namespace {

// Size classes: 4 KiB granularity below 1 MiB, then quarter-power-of-two
// steps, so a recycled block wastes at most ~19 % and repeated frames of one
// geometry always hit the same class.
size_t size_class(size_t n) {
    if (n <= (1u << 20)) return (n + 4095) & ~size_t(4095);
    size_t p = 1u << 20;
    while (p < n) p <<= 1;
    const size_t q = p >> 3;  // 8 steps between p/2 and p
    size_t s = p >> 1;
    while (s < n) s += q;
    return s;
}

// Unused blocks kept per pool before freeing (host pinned / device HBM).
constexpr size_t kHostCacheCap = size_t(2) << 30;
constexpr size_t kDeviceCacheCap = size_t(16) << 30;

struct Pool {
    std::mutex mu;
    std::multimap<size_t, void*> free_blocks;  // class -> block
    std::unordered_map<void*, size_t> live;    // block -> class
    size_t cached = 0;
};

enum HostMode { kUnknown, kPinned, kPageable };

struct HostPool : Pool {
    HostMode mode = kUnknown;
};

HostPool& host_pool() {
    static HostPool* p = new HostPool;  // never destroyed: blocks may outlive static teardown
    return *p;
}

std::mutex g_dev_mu;
std::map<int, Pool*>& device_pools() {
    static auto* m = new std::map<int, Pool*>;
    return *m;
}

Pool& device_pool(int device) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    Pool*& p = device_pools()[device];
    if (!p) p = new Pool;
    return *p;
}

HostMode host_mode(HostPool& hp) {
    if (hp.mode == kUnknown) {
        const char* env = std::getenv("VACV_PINNED_HOST");
        int n = 0;
        const bool gpu = hipGetDeviceCount(&n) == hipSuccess && n > 0;
        hp.mode = (gpu && !(env && env[0] == '0')) ? kPinned : kPageable;
    }
    return hp.mode;
}

void* raw_host_alloc(HostMode mode, size_t n) {
    void* p = nullptr;
    if (mode == kPinned) {
        if (hipHostMalloc(&p, n, hipHostMallocDefault) == hipSuccess) return p;
        return nullptr;
    }
    if (posix_memalign(&p, 64, n) != 0) return nullptr;
    return p;
}

void raw_host_free(HostMode mode, void* p) {
    if (mode == kPinned) {
        (void)hipHostFree(p);
    } else {
        std::free(p);
    }
}

// Take a cached block of class `cls`, or nullptr.
void* take(Pool& pool, size_t cls) {
    auto it = pool.free_blocks.find(cls);
    if (it == pool.free_blocks.end()) return nullptr;
    void* p = it->second;
    pool.free_blocks.erase(it);
    pool.cached -= cls;
    pool.live[p] = cls;
    return p;
}

}  // namespace

void* VaAllocator::allocate(size_t len) {
    if (len == 0) return nullptr;
    HostPool& hp = host_pool();
    std::lock_guard<std::mutex> lk(hp.mu);
    const HostMode mode = host_mode(hp);
    const size_t cls = size_class(len);
    if (void* p = take(hp, cls)) return p;
    void* p = raw_host_alloc(mode, cls);
    if (!p && !hp.free_blocks.empty()) {  // pinned memory exhausted: drop the cache, retry once
        for (auto& kv : hp.free_blocks) raw_host_free(mode, kv.second);
        hp.free_blocks.clear();
        hp.cached = 0;
        p = raw_host_alloc(mode, cls);
    }
    if (p) hp.live[p] = cls;
    return p;
}

void VaAllocator::deallocate(void* ptr) {
    if (!ptr) return;
    HostPool& hp = host_pool();
    std::lock_guard<std::mutex> lk(hp.mu);
    auto it = hp.live.find(ptr);
    if (it == hp.live.end()) return;  // not ours (a view): nothing to free
    const size_t cls = it->second;
    hp.live.erase(it);
    if (hp.cached + cls <= kHostCacheCap) {
        hp.free_blocks.emplace(cls, ptr);
        hp.cached += cls;
    } else {
        raw_host_free(hp.mode, ptr);
    }
}

void* VaAllocator::allocate_device(size_t len, int device) {
    if (len == 0 || device < 0) return nullptr;
    Pool& pool = device_pool(device);
    std::lock_guard<std::mutex> lk(pool.mu);
    const size_t cls = size_class(len);
    if (void* p = take(pool, cls)) return p;
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) return nullptr;
    if (prev != device && hipSetDevice(device) != hipSuccess) return nullptr;
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, cls);
    if (e != hipSuccess && !pool.free_blocks.empty()) {
        (void)hipGetLastError();
        for (auto& kv : pool.free_blocks) (void)hipFree(kv.second);
        pool.free_blocks.clear();
        pool.cached = 0;
        e = hipMalloc(&p, cls);
    }
    if (prev != device) (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    pool.live[p] = cls;
    return p;
}

void VaAllocator::deallocate_device(void* ptr, int device) {
    if (!ptr || device < 0) return;
    Pool& pool = device_pool(device);
    std::lock_guard<std::mutex> lk(pool.mu);
    auto it = pool.live.find(ptr);
    if (it == pool.live.end()) return;
    const size_t cls = it->second;
    pool.live.erase(it);
    if (pool.cached + cls <= kDeviceCacheCap) {
        pool.free_blocks.emplace(cls, ptr);
        pool.cached += cls;
    } else {
        (void)hipFree(ptr);  // hipFree waits for work still using the block
    }
}

size_t VaAllocator::align_size(size_t sz, size_t n) { return (sz + n - 1) & ~(n - 1); }

bool VaAllocator::host_pinned() {
    HostPool& hp = host_pool();
    std::lock_guard<std::mutex> lk(hp.mu);
    return host_mode(hp) == kPinned;
}

void VaAllocator::trim() {
    {
        HostPool& hp = host_pool();
        std::lock_guard<std::mutex> lk(hp.mu);
        for (auto& kv : hp.free_blocks) raw_host_free(hp.mode, kv.second);
        hp.free_blocks.clear();
        hp.cached = 0;
    }
    std::lock_guard<std::mutex> lk(g_dev_mu);
    for (auto& d : device_pools()) {
        std::lock_guard<std::mutex> lk2(d.second->mu);
        for (auto& kv : d.second->free_blocks) (void)hipFree(kv.second);
        d.second->free_blocks.clear();
        d.second->cached = 0;
    }
}

size_t VaAllocator::cached_host_bytes() {
    HostPool& hp = host_pool();
    std::lock_guard<std::mutex> lk(hp.mu);
    return hp.cached;
}

size_t VaAllocator::cached_device_bytes() {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    size_t t = 0;
    for (auto& d : device_pools()) {
        std::lock_guard<std::mutex> lk2(d.second->mu);
        t += d.second->cached;
    }
    return t;
}

}  // namespace vision
