// Kernel launch checks (hip_launch.hpp).
#include "hip_launch.hpp"

#include <cstdio>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>

namespace madrona::hipx {

void hipFail(hipError_t err, const char *expr, const char *file, int line)
{
    std::fprintf(stderr, "HIP error %s at %s:%d (%s)\n", hipGetErrorString(err), file, line, expr);
    throw std::runtime_error(std::string(hipGetErrorString(err)) + " (" + expr + ")");
}

namespace {

struct Shape {
    int32_t dev;
    const void *fn;
    int32_t threads;
    size_t lds;
    bool operator<(const Shape &o) const
    {
        return std::tie(dev, fn, threads, lds) < std::tie(o.dev, o.fn, o.threads, o.lds);
    }
};

struct Verdict {
    int32_t blocks;          // resident blocks per CU, 0: cannot launch
    std::string why;         // reason when blocks == 0
};

std::mutex g_mu;
std::map<Shape, Verdict> g_cache;
std::map<int32_t, size_t> g_maxLDS;

size_t deviceMaxLDS(int32_t dev)
{
    auto it = g_maxLDS.find(dev);
    if (it != g_maxLDS.end()) return it->second;
    int v = 0;
    MW_HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
    g_maxLDS[dev] = (size_t)v;
    return (size_t)v;
}

Verdict evaluate(int32_t dev, const void *fn, int32_t threads, size_t dyn_lds)
{
    hipFuncAttributes attr {};
    MW_HIP_CHECK(hipFuncGetAttributes(&attr, fn));
    const size_t limit = deviceMaxLDS(dev);
    const size_t total = attr.sharedSizeBytes + dyn_lds;
    char buf[256];
    if (threads <= 0 || threads > attr.maxThreadsPerBlock) {
        std::snprintf(buf, sizeof(buf), "%d lanes per block, the kernel's bound is %d", threads,
                      attr.maxThreadsPerBlock);
        return { 0, buf };
    }
    if (total > limit) {
        std::snprintf(buf, sizeof(buf),
                      "%zu B of LDS per block (%zu static + %zu dynamic) exceed the device's %zu B",
                      total, (size_t)attr.sharedSizeBytes, dyn_lds, limit);
        return { 0, buf };
    }
    int per_cu = 0;
    MW_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, dyn_lds));
    if (per_cu <= 0) {
        std::snprintf(buf, sizeof(buf),
                      "no block of %d lanes with %zu B of LDS (%zu static + %zu dynamic) and %d "
                      "VGPR-spill bytes fits a CU",
                      threads, total, (size_t)attr.sharedSizeBytes, dyn_lds, (int)attr.localSizeBytes);
        return { 0, buf };
    }
    return { per_cu, {} };
}

const Verdict &lookup(const void *fn, int32_t threads, size_t dyn_lds)
{
    int dev = 0;
    MW_HIP_CHECK(hipGetDevice(&dev));
    const Shape key { dev, fn, threads, dyn_lds };
    auto it = g_cache.find(key);
    if (it != g_cache.end()) return it->second;
    return g_cache.emplace(key, evaluate(dev, fn, threads, dyn_lds)).first->second;
}

}

size_t maxLDSPerBlock()
{
    std::lock_guard<std::mutex> lk(g_mu);
    int dev = 0;
    MW_HIP_CHECK(hipGetDevice(&dev));
    return deviceMaxLDS(dev);
}

int32_t residentBlocksNoThrow(const void *fn, int32_t threads, size_t dyn_lds)
{
    std::lock_guard<std::mutex> lk(g_mu);
    return lookup(fn, threads, dyn_lds).blocks;
}

int32_t residentBlocks(const void *fn, const char *name, int32_t threads, size_t dyn_lds)
{
    std::lock_guard<std::mutex> lk(g_mu);
    const Verdict &v = lookup(fn, threads, dyn_lds);
    if (v.blocks > 0) return v.blocks;
    const std::string msg = std::string("kernel ") + name + " cannot launch: " + v.why;
    std::fprintf(stderr, "%s\n", msg.c_str());
    throw std::runtime_error(msg);
}

void checkLaunched(const char *name)
{
    const hipError_t err = hipGetLastError();
    if (err == hipSuccess) return;
    const std::string msg = std::string("kernel ") + name + " launch failed: " + hipGetErrorString(err);
    std::fprintf(stderr, "%s\n", msg.c_str());
    throw std::runtime_error(msg);
}

}
