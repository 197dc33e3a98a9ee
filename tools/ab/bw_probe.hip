// Read-bandwidth probe (timing experiments only): where K1's memory bound sits.
// One 512-thread workgroup per CU streams a 4 GiB buffer in 128 KiB rounds (16 x 16 B loads per
// thread in flight, like K1's tile), grid-stride over rounds.  Workgroups are filtered by their
// dispatch index (workgroup i runs on XCD i mod 8): all, the even ones (4 XCDs, every CU), or
// i mod 16 < 8 (every XCD, half its CUs).  Equal rates for the last two = a per-XCD (or global)
// cap; a rate proportional to the active CUs = a per-CU cap.
// build: hipcc -O3 --offload-arch=gfx950 tools/ab/bw_probe.hip -o /tmp/bw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512, 1) void k_read(const u32x4* __restrict__ in, size_t n16, int mode, unsigned* out) {
    const int b = blockIdx.x;
    if ((mode == 1 && (b & 1)) || (mode == 2 && (b & 15) >= 8)) return;
    const size_t per = 512 * 16;   // 16-B units per round
    const size_t rounds = n16 / per;
    // rank among the active workgroups: they stride over every round of the buffer
    const int rank = mode == 0 ? b : mode == 1 ? b / 2 : (b / 16) * 8 + (b & 15);
    const int nact = mode == 0 ? (int)gridDim.x : (int)gridDim.x / 2;
    u32x4 acc = {0, 0, 0, 0};
    for (size_t r = rank; r < rounds; r += nact) {
        const u32x4* p = in + r * per + threadIdx.x;
        u32x4 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = __builtin_nontemporal_load(p + u * 512);
#pragma unroll
        for (int u = 0; u < 16; ++u) acc ^= v[u];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;   // keeps the loads
}

int main() {
    const size_t bytes = (size_t)4 << 30, n16 = bytes / 16;
    void* d;
    unsigned* o;
    if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&o, 4) != hipSuccess) return 1;
    hipMemset(d, 1, bytes);
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[3] = {"all CUs", "even workgroups (4 XCDs, all their CUs)", "i mod 16 < 8 (8 XCDs, half the CUs)"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 3; ++mode) {
            hipLaunchKernelGGL(k_read, dim3(ncu), dim3(512), 0, 0, (const u32x4*)d, n16, mode, o);
            hipEventRecord(e0, 0);
            for (int it = 0; it < 5; ++it)
                hipLaunchKernelGGL(k_read, dim3(ncu), dim3(512), 0, 0, (const u32x4*)d, n16, mode, o);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            // every mode reads the whole buffer: the active workgroups stride over all rounds
            printf("%d %-44s %7.1f GB/s\n", rep, names[mode], 5.0 * bytes / (ms * 1e-3) / 1e9);
        }
    return 0;
}
