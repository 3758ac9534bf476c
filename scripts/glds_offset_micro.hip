// Semantics check of global_load_lds_dwordx4's instruction offset on gfx950:
// is `offset:` added to the global address only, or to the LDS address too?
// One wave: M0 = 0, v = lane*16, offset:1024; the LDS image is copied out and
// compared against the source (src[i] = i).  Prints which addresses were used.
//   hipcc --offload-arch=gfx950 -O2 scripts/glds_offset_micro.hip -o scripts/glds_offset_micro.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(64) void k(const float *__restrict__ src, float *__restrict__ out)
{
    __shared__ __attribute__((aligned(16))) float lds[2048];
    const int lane = threadIdx.x;
    for (int i = lane; i < 2048; i += 64) lds[i] = -1.0f;
    __syncthreads();
    const float *g = src + lane * 4;  // lane*16 bytes
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\t"
                 "s_mov_b32 m0, 0\n\t"
                 "s_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off offset:1024\n\t"
                 "s_waitcnt vmcnt(0)\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g)
                 : "memory");
    __syncthreads();
    for (int i = lane; i < 2048; i += 64) out[i] = lds[i];
}

int main()
{
    std::vector<float> h(4096);
    for (int i = 0; i < 4096; i++) h[i] = (float)i;
    float *src, *out;
    hipMalloc(&src, 4096 * 4);
    hipMalloc(&out, 2048 * 4);
    hipMemcpy(src, h.data(), 4096 * 4, hipMemcpyHostToDevice);
    k<<<1, 64>>>(src, out);
    std::vector<float> o(2048);
    hipMemcpy(o.data(), out, 2048 * 4, hipMemcpyDeviceToHost);
    // where did lane 0's 16 bytes land, and which source bytes are they?
    int first = -1;
    for (int i = 0; i < 2048; i++)
        if (o[i] >= 0) {
            first = i;
            break;
        }
    printf("first written LDS dword %d (byte %d) holds src dword %.0f (byte %.0f)\n", first, first * 4,
           first >= 0 ? o[first] : -1.f, first >= 0 ? o[first] * 4 : -1.f);
    int written = 0;
    for (int i = 0; i < 2048; i++) written += o[i] >= 0;
    printf("dwords written: %d\n", written);
    const bool lds_too = first == 256 && o[256] == 256.f;
    const bool global_only = first == 0 && o[0] == 256.f;
    printf("offset applies to: %s\n", lds_too ? "global AND LDS" : global_only ? "global only" : "other");
    return 0;
}
