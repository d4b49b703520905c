// managed_probe.hip — where hipMallocManaged memory lives on this box and how fast a kernel and the
// copy engines reach it (the reference allocates its image as cudaMallocManaged, Core/image.cpp:15-27).
//   hipcc --offload-arch=gfx950 -O2 tools/managed_probe.hip -o /tmp/managed_probe && /tmp/managed_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void rmw(float4* a, size_t n) {  // read-modify-write stream, like the accumulate kernel
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        v.x += 1.0f;
        a[i] = v;
    }
}

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
    const size_t bytes = (size_t)1920 * 1080 * 12;  // the metric frame's float3 running sum
    const size_t n4 = bytes / 16;
    int dev = 0, v = 0;
    CK(hipGetDevice(&dev));
    const hipDeviceAttribute_t attrs[] = {hipDeviceAttributeManagedMemory, hipDeviceAttributeConcurrentManagedAccess,
                                          hipDeviceAttributePageableMemoryAccess,
                                          hipDeviceAttributePageableMemoryAccessUsesHostPageTables,
                                          hipDeviceAttributeDirectManagedMemAccessFromHost};
    const char* names[] = {"ManagedMemory", "ConcurrentManagedAccess", "PageableMemoryAccess",
                           "PageableMemoryAccessUsesHostPageTables", "DirectManagedMemAccessFromHost"};
    for (int i = 0; i < 5; i++) {
        v = -1;
        (void)hipDeviceGetAttribute(&v, attrs[i], dev);
        std::printf("attr %-40s %d\n", names[i], v);
    }
    void* m = nullptr;
    CK(hipMallocManaged(&m, bytes, hipMemAttachGlobal));
    hipPointerAttribute_t pa;
    CK(hipPointerGetAttributes(&pa, m));
    std::printf("managed: type %d (device %d, host %d, array %d, unified %d, managed %d), isManaged %d, device %d\n",
                (int)pa.type, (int)hipMemoryTypeDevice, (int)hipMemoryTypeHost, (int)hipMemoryTypeArray,
                (int)hipMemoryTypeUnified, (int)hipMemoryTypeManaged, pa.isManaged, pa.device);
    void* d = nullptr;
    CK(hipMalloc(&d, bytes));
    void* h = nullptr;
    CK(hipHostMalloc(&h, bytes, 0));
    std::vector<char> pageable(bytes);
    hipStream_t s;
    CK(hipStreamCreate(&s));
    auto host_touch = [&](void* p, const char* what) {
        auto t = std::chrono::steady_clock::now();
        std::memset(p, 0, bytes);
        std::printf("host memset %-10s %8.3f ms\n", what, ms_since(t));
        t = std::chrono::steady_clock::now();
        volatile float acc = 0.0f;
        const float* f = (const float*)p;
        for (size_t i = 0; i < bytes / 4; i += 16) acc += f[i];
        std::printf("host read   %-10s %8.3f ms\n", what, ms_since(t));
    };
    host_touch(m, "managed");
    host_touch(h, "pinned");
    for (int rep = 0; rep < 3; rep++) {
        for (int which = 0; which < 3; which++) {
            void* p = which == 0 ? m : (which == 1 ? d : h);
            CK(hipStreamSynchronize(s));
            auto t = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(rmw, dim3(4096), dim3(256), 0, s, (float4*)p, n4);
            CK(hipGetLastError());
            CK(hipStreamSynchronize(s));
            std::printf("kernel rmw %-8s rep %d %8.3f ms (%.1f GB/s)\n", which == 0 ? "managed" : (which == 1 ? "device" : "pinned"),
                        rep, ms_since(t), 2.0 * bytes / ms_since(t) / 1e6);
        }
        host_touch(m, "managed");  // the CPU twin writes the image between GPU passes
    }
    struct C { void* dst; const void* src; const char* what; } copies[] = {
        {d, m, "managed->device"}, {m, d, "device->managed"}, {d, pageable.data(), "pageable->device"},
        {pageable.data(), d, "device->pageable"}, {d, h, "pinned->device"}, {h, d, "device->pinned"}};
    for (int rep = 0; rep < 2; rep++)
        for (const C& c : copies) {
            auto t = std::chrono::steady_clock::now();
            CK(hipMemcpyAsync(c.dst, c.src, bytes, hipMemcpyDefault, s));
            CK(hipStreamSynchronize(s));
            std::printf("copy %-18s rep %d %8.3f ms (%.1f GB/s)\n", c.what, rep, ms_since(t), bytes / ms_since(t) / 1e6);
        }
    CK(hipFree(m)); CK(hipFree(d)); CK(hipHostFree(h));
    return 0;
}
