// ell_micro.hip -- diagnostic micro-benchmark for the small-M walk
// (csrc/tsg_ell.hip): cycles per entry of ONE column chain per lane, by
// addressing mode, with the real kernel's structure (16-byte index blocks of
// 8 uint16 entries prefetched 32 deep, the LDS reads of block d+1 issued
// between the adds of block d).  Not part of the library; built and run by
// scripts/ell_micro.sh.  Wave-cycles come from s_memtime stamps outside the
// walk (a diagnostic build: read the ratios, not absolute kernel times).
//
// modes: 0 float index, C++ addressing (and/bfe + lshl_add: 2 VALU / entry)
//        1 float index, v_mad_u32_u16 op_sel addressing (1 VALU / entry)
//        2 no LDS read (the index itself as the addend: VALU + stream only)
//        3 mode 1 with 4 rows per lane (ds_read_b128 + 4 independent adds)
//        4 mode 1 with 2 rows per lane (ds_read_b64 + 2 adds)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

typedef __attribute__((address_space(3))) const float lds_f;
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const v2f lds_f2;
typedef __attribute__((address_space(3))) const v4f lds_f4;

__device__ __forceinline__ uint32_t mad_lo(uint32_t w, uint32_t base)
{
    uint32_t r;
    asm("v_mad_u32_u16 %0, %1, 4, %2" : "=v"(r) : "v"(w), "v"(base));
    return r;
}
__device__ __forceinline__ uint32_t mad_hi(uint32_t w, uint32_t base)
{
    uint32_t r;
    asm("v_mad_u32_u16 %0, %1, 4, %2 op_sel:[1,0,0,0]" : "=v"(r) : "v"(w), "v"(base));
    return r;
}

template <int MODE> struct Rows { static constexpr int R = MODE == 3 ? 4 : MODE == 4 ? 2 : 1; };
// mode 5: mode 1 + ONE s_waitcnt lgkmcnt(8) per block before its adds

template <int MODE>
__device__ __forceinline__ void load8(float (&x)[8][Rows<MODE>::R], const uint4 e, const float *xs, uint32_t base)
{
    constexpr int R = Rows<MODE>::R;
    const uint32_t w[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
    for (int h = 0; h < 8; h++) {
        const uint32_t ww = w[h >> 1];
        if constexpr (MODE == 0) {
            x[h][0] = xs[(ww >> (16 * (h & 1))) & 0xffffu];
        } else if constexpr (MODE == 2) {
            x[h][0] = __uint_as_float((ww >> (16 * (h & 1))) & 0xffffu);
        } else {
            const uint32_t a = (h & 1) ? mad_hi(ww, base) : mad_lo(ww, base);
            if constexpr (R == 1) x[h][0] = *(lds_f *)(uintptr_t)a;
            else if constexpr (R == 2) {
                const v2f v = *(lds_f2 *)(uintptr_t)a;
                x[h][0] = v.x; x[h][1] = v.y;
            } else {
                const v4f v = *(lds_f4 *)(uintptr_t)a;
                x[h][0] = v.x; x[h][1] = v.y; x[h][2] = v.z; x[h][3] = v.w;
            }
        }
    }
}

template <int MODE>
__device__ __forceinline__ void add8(float (&y)[Rows<MODE>::R], const float (&x)[8][Rows<MODE>::R])
{
#pragma unroll
    for (int h = 0; h < 8; h++)
#pragma unroll
        for (int r = 0; r < Rows<MODE>::R; r++) y[r] += x[h][r];
}

template <int MODE, bool SB, int ACT>
__global__ __launch_bounds__(64) void walk(const uint4 *__restrict__ ent, int nblk, int ncol, float *out,
                                           unsigned long long *cyc)
{
    constexpr int R = Rows<MODE>::R, D = 32;
    extern __shared__ __attribute__((aligned(16))) float xs[];  // 4096 * R floats
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096 * R; i += 64) xs[i] = (float)(i % 97) * 0.25f;
    __syncthreads();
    const uint32_t base = (uint32_t)(uintptr_t)(lds_f *)xs;
    const int col = blockIdx.x * 64 + lane;
    const uint4 *p = ent + col;
    float y[R];
#pragma unroll
    for (int r = 0; r < R; r++) y[r] = 0.0f;
    unsigned long long t0, t1;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    if (lane < ACT) {
    const uint32_t last = nblk - 1;
    uint4 q[D];
#pragma unroll
    for (int d = 0; d < D; d++) q[d] = p[(size_t)min((uint32_t)d, last) * ncol];
    for (uint32_t i = 0; i + D <= (uint32_t)nblk; i += D) {
        float x0[8][R], x1[8][R];
        load8<MODE>(x0, q[0], xs, base);
#pragma unroll
        for (int d = 0; d < D; d++) {
            if (d + 1 < D) {
                if (d % 2 == 0) load8<MODE>(x1, q[d + 1], xs, base);
                else load8<MODE>(x0, q[d + 1], xs, base);
            }
            if (SB) __builtin_amdgcn_sched_barrier(0);  // block d+1's reads stay ahead of block d's adds
            if (MODE == 5) {
                if (d + 1 < D) __builtin_amdgcn_s_waitcnt(0xC87F);  // lgkmcnt(8)
                else __builtin_amdgcn_s_waitcnt(0xC07F);            // lgkmcnt(0)
            }
            add8<MODE>(y, d % 2 == 0 ? x0 : x1);
            if (SB) __builtin_amdgcn_sched_barrier(0);
            q[d] = p[(size_t)min(i + D + d, last) * ncol];
        }
    }
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    float s = 0.0f;
#pragma unroll
    for (int r = 0; r < R; r++) s += y[r];
    out[col] = s;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, bool SB = true, int ACT = 64>
void run(const uint4 *dent, int nblk, int ncol, float *dout, unsigned long long *dcyc, int grid)
{
    constexpr int R = Rows<MODE>::R;
    const size_t lds = 4096 * R * sizeof(float);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 30; w++) hipLaunchKernelGGL((walk<MODE, SB, ACT>), dim3(grid), dim3(64), lds, 0, dent, nblk, ncol, dout, dcyc);
    CK(hipEventRecord(a));
    const int reps = 20;
    for (int w = 0; w < reps; w++) hipLaunchKernelGGL((walk<MODE, SB, ACT>), dim3(grid), dim3(64), lds, 0, dent, nblk, ncol, dout, dcyc);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<unsigned long long> c(grid);
    CK(hipMemcpy(c.data(), dcyc, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double avg = 0;
    for (auto v : c) avg += (double)v;
    avg /= grid;
    const double entries = nblk * 8.0;
    std::printf("mode %d sb %d act %2d rows %d grid %5d nblk %4d: kernel %.2f us, %.1f ns/entry, stamp %.1f memtime-ticks/entry\n",
                MODE, (int)SB, ACT, R, grid, nblk, ms * 1000.0 / reps, ms * 1e6 / reps / entries, avg / entries);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}


// DPP chain: G lanes per column gather G consecutive entries with ONE LDS read
// each; every lane of the column then adds the G values in entry order,
// broadcast within the column's lanes by DPP (row_newbcast for G = 16,
// quad_perm for G = 4), so each chain step is one v_add_f32_dpp.
template <int G, int I>
__device__ __forceinline__ float bcast(float x)
{
    constexpr int ctrl = G == 16 ? 0x150 + I : I * 0x55;  // row_newbcast:I / quad_perm:[I,I,I,I]
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), ctrl, 0xf, 0xf, true));
}
// y += x(lane 0) + ... in lane order: entries 0..G-1 of the group
template <int G, int I> struct Chain {
    static __device__ __forceinline__ void run(float &y, float x)
    {
        Chain<G, I - 1>::run(y, x);
        y += bcast<G, I - 1>(x);
    }
};
template <int G> struct Chain<G, 0> {
    static __device__ __forceinline__ void run(float &, float) {}
};

template <int G>
__global__ __launch_bounds__(64) void walk_dpp(const uint4 *__restrict__ ent, int nblk, float *out,
                                               unsigned long long *cyc)
{
    constexpr int D = 8;  // 16-byte loads in flight per lane (8 entries each)
    extern __shared__ __attribute__((aligned(16))) float xs[];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096; i += 64) xs[i] = (float)(i % 97) * 0.25f;
    __syncthreads();
    const uint32_t base = (uint32_t)(uintptr_t)(lds_f *)xs;
    const int col = blockIdx.x * (64 / G) + lane / G, g = lane % G;
    // block t of the column: G lanes x 8 entries (entry 8G t + G j + g in lane g, slot j)
    const uint4 *p = ent + (size_t)col * nblk * G + g;
    float y = 0.0f;
    unsigned long long t0, t1;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    uint4 q[D];
#pragma unroll
    for (int d = 0; d < D; d++) q[d] = p[(size_t)min(d, nblk - 1) * G];
    for (int t = 0; t < nblk; t += D) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            const uint32_t w[4] = {q[d].x, q[d].y, q[d].z, q[d].w};
            float x[8];
#pragma unroll
            for (int j = 0; j < 8; j++)
                x[j] = *(lds_f *)(uintptr_t)((j & 1) ? mad_hi(w[j >> 1], base) : mad_lo(w[j >> 1], base));
            q[d] = p[(size_t)min(t + D + d, nblk - 1) * G];
#pragma unroll
            for (int j = 0; j < 8; j++) Chain<G, G>::run(y, x[j]);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    if (g == 0) out[col] = y;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int G>
void run_dpp(const uint4 *dent, int nblk, float *dout, unsigned long long *dcyc, int grid)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 30; w++) hipLaunchKernelGGL(walk_dpp<G>, dim3(grid), dim3(64), 16384, 0, dent, nblk, dout, dcyc);
    CK(hipEventRecord(a));
    const int reps = 20;
    for (int w = 0; w < reps; w++) hipLaunchKernelGGL(walk_dpp<G>, dim3(grid), dim3(64), 16384, 0, dent, nblk, dout, dcyc);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<unsigned long long> c(grid);
    CK(hipMemcpy(c.data(), dcyc, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double avg = 0;
    for (auto v : c) avg += (double)v;
    avg /= grid;
    const double entries = nblk * 8.0 * G;
    std::printf("dpp G %2d grid %5d (%6d columns) entries/col %5.0f: kernel %.2f us, %.2f ns/entry, stamp %.2f ticks/entry\n",
                G, grid, grid * 64 / G, entries, ms * 1000.0 / reps, ms * 1e6 / reps / entries, avg / entries);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

// Producer / consumer: P producer waves gather the X values of the next phase
// (E entries of each of 64 columns) into an LDS buffer in chain order while
// the consumer wave (lane = column) adds the current phase's from the other
// buffer, 4 per ds_read_b128; one barrier per phase.
// a workgroup barrier that orders LDS only (global loads stay in flight)
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int E>
__global__ __launch_bounds__(64 * (1 + E / 8)) void walk_pc(const uint4 *__restrict__ ent, int nblk, float *out,
                                                            unsigned long long *cyc)
{
    constexpr int P = E / 8, D = 16;  // producer waves; phases of index blocks in flight per producer lane
    __shared__ __attribute__((aligned(16))) float xs[4096];
    __shared__ __attribute__((aligned(16))) float4 buf[2][E / 4][64];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (int i = tid; i < 4096; i += 64 * (1 + P)) xs[i] = (float)(i % 97) * 0.25f;
    const uint32_t base = (uint32_t)(uintptr_t)(lds_f *)xs;
    const int nph = nblk * 8 / E;
    const int col0 = blockIdx.x * 64;
    __syncthreads();
    unsigned long long t0 = 0, t1 = 0;
    if (wave == 0) {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
        __builtin_amdgcn_sched_barrier(0);
    }
    if (wave == 0) {  // consumer
        float y = 0.0f;
        lds_barrier();  // phase 0 filled
        for (int ph = 0; ph < nph; ph++) {
            const float4 *bp = &buf[ph & 1][0][lane];
#pragma unroll
            for (int q4 = 0; q4 < E / 4; q4++) {
                const float4 v = bp[q4 * 64];
                y += v.x; y += v.y; y += v.z; y += v.w;
            }
            lds_barrier();
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
        __builtin_amdgcn_sched_barrier(0);
        out[col0 + lane] = y;
        if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    } else {  // producer: column lane, block j of each phase
        const int j = wave - 1;
        const uint4 *p = ent + (size_t)j * 65536 + col0 + lane;  // block ph * P + j of the column: lanes contiguous
        uint4 q[D];
#pragma unroll
        for (int d = 0; d < D; d++) q[d] = p[(size_t)min(d, nph - 1) * P * 65536];
        auto fill = [&](int ph, const uint4 e) {
            const uint32_t w[4] = {e.x, e.y, e.z, e.w};
            float x[8];
#pragma unroll
            for (int h = 0; h < 8; h++)
                x[h] = *(lds_f *)(uintptr_t)((h & 1) ? mad_hi(w[h >> 1], base) : mad_lo(w[h >> 1], base));
            buf[ph & 1][2 * j][lane] = make_float4(x[0], x[1], x[2], x[3]);
            buf[ph & 1][2 * j + 1][lane] = make_float4(x[4], x[5], x[6], x[7]);
        };
        fill(0, q[0]);
        q[0] = p[(size_t)min(D, nph - 1) * P * 65536];
        lds_barrier();
        // branch-free: phase g + d + 1 from slot (d + 1) % D (the last fill,
        // phase nph, lands in the buffer nobody reads again)
        for (int g = 0; g < nph; g += D) {
#pragma unroll
            for (int d = 0; d < D; d++) {
                const int ph = g + d + 1;
                fill(ph, q[(d + 1) % D]);
                q[(d + 1) % D] = p[(size_t)min(ph + D, nph - 1) * P * 65536];
                lds_barrier();
            }
        }
    }
}

template <int E>
void run_pc(const uint4 *dent, int nblk, float *dout, unsigned long long *dcyc, int grid)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 30; w++) hipLaunchKernelGGL(walk_pc<E>, dim3(grid), dim3(64 * (1 + E / 8)), 0, 0, dent, nblk, dout, dcyc);
    CK(hipEventRecord(a));
    const int reps = 20;
    for (int w = 0; w < reps; w++) hipLaunchKernelGGL(walk_pc<E>, dim3(grid), dim3(64 * (1 + E / 8)), 0, 0, dent, nblk, dout, dcyc);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<unsigned long long> c(grid);
    CK(hipMemcpy(c.data(), dcyc, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double avg = 0;
    for (auto v : c) avg += (double)v;
    avg /= grid;
    const double entries = nblk * 8.0;
    std::printf("pc E %2d grid %5d (%6d columns) entries/col %5.0f: kernel %.2f us, %.2f ns/entry, stamp %.2f ticks/entry\n",
                E, grid, grid * 64, entries, ms * 1000.0 / reps, ms * 1e6 / reps / entries, avg / entries);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

// The consumer's floor: CH independent chains per lane, fed 4 values per
// ds_read_b128 from a lane-contiguous LDS buffer (no gather, no barrier).
template <int CH>
__global__ __launch_bounds__(64) void chain_floor(int n4, float *out, unsigned long long *cyc)
{
    __shared__ __attribute__((aligned(16))) float4 buf[64][64];
    const int lane = threadIdx.x;
    for (int i = 0; i < 64; i++) buf[i][lane] = make_float4(lane, i, 0.5f, 0.25f);
    __syncthreads();
    float y[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) y[c] = 0.0f;
    unsigned long long t0, t1;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    for (int i = 0; i < n4; i += 16) {
        float4 v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = buf[(i + u) & 63][lane];
#pragma unroll
        for (int u = 0; u < 16; u++) {
            if constexpr (CH == 1) { y[0] += v[u].x; y[0] += v[u].y; y[0] += v[u].z; y[0] += v[u].w; }
            else if constexpr (CH == 2) { y[0] += v[u].x; y[1] += v[u].y; y[0] += v[u].z; y[1] += v[u].w; }
            else { y[0] += v[u].x; y[1] += v[u].y; y[2] += v[u].z; y[3] += v[u].w; }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < CH; c++) s += y[c];
    out[blockIdx.x * 64 + lane] = s;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CH>
void run_floor(float *dout, unsigned long long *dcyc)
{
    const int n4 = 1024;  // 4096 adds per lane
    for (int w = 0; w < 10; w++) hipLaunchKernelGGL(chain_floor<CH>, dim3(4), dim3(64), 0, 0, n4, dout, dcyc);
    CK(hipDeviceSynchronize());
    unsigned long long c[4];
    CK(hipMemcpy(c, dcyc, sizeof(c), hipMemcpyDeviceToHost));
    std::printf("chain floor: %d chains per lane, %.2f ticks per add (%.2f per add of one chain)\n", CH,
                (double)c[0] / (4.0 * n4), (double)c[0] / (4.0 * n4) * CH);
}

int main()
{
    const int ncol = 1024 * 64;  // up to 1024 waves
    const int nblk = 128;        // 1024 entries per chain (BaseTCSC K/s at K=4096, s=4)
    std::vector<uint32_t> h((size_t)nblk * ncol * 4);
    uint32_t s = 12345;
    for (auto &v : h) {
        s = s * 1664525u + 1013904223u;
        const uint32_t lo = (s >> 4) % 4096, hi = (s >> 18) % 4096;
        v = lo * 4 | (hi * 4) << 16;  // float index of a row with 4 floats (valid for every R)
    }
    // for R = 1 the index (< 16384) addresses 4096 * R floats only if < 4096: rescale
    std::vector<uint32_t> h1(h);
    for (auto &v : h1) v = ((v & 0xffffu) / 4) | (((v >> 16) / 4) << 16);
    std::vector<uint32_t> h2(h);
    for (auto &v : h2) v = ((v & 0xffffu) / 2) | (((v >> 16) / 2) << 16);
    uint4 *d1, *d2, *d4;
    float *dout;
    unsigned long long *dcyc;
    CK(hipMalloc(&d1, h.size() * 4));
    CK(hipMalloc(&d2, h.size() * 4));
    CK(hipMalloc(&d4, h.size() * 4));
    CK(hipMalloc(&dout, 65536 * sizeof(float)));
    CK(hipMalloc(&dcyc, 4096 * sizeof(unsigned long long)));
    CK(hipMemcpy(d1, h1.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d2, h2.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d4, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    // DPP chains: 1024 entries per column; d1 holds >= 4096 * 64 * 128 * 4 words
    run_floor<1>(dout, dcyc);
    run_floor<2>(dout, dcyc);
    run_floor<4>(dout, dcyc);
    for (int grid : {4, 256, 1024}) {
        run_pc<16>(d1, 128, dout, dcyc, grid);
        run_pc<32>(d1, 128, dout, dcyc, grid);
        run<1>(d1, 128, ncol, dout, dcyc, grid);
        run<5>(d1, 128, ncol, dout, dcyc, grid);
        run<1, true, 16>(d1, 128, ncol, dout, dcyc, grid);
        run<5, true, 16>(d1, 128, ncol, dout, dcyc, grid);
        if (grid <= 1024) run_dpp<4>(d1, 32, dout, dcyc, grid);
    }
    if (getenv("ELL_MICRO_ALL") == nullptr) return 0;
    for (int grid : {4, 256, 1024}) {
        for (int nb : {128}) {
            run<0, false>(d1, nb, ncol, dout, dcyc, grid);
            run<0>(d1, nb, ncol, dout, dcyc, grid);
            run<1, false>(d1, nb, ncol, dout, dcyc, grid);
            run<1>(d1, nb, ncol, dout, dcyc, grid);
            run<2>(d1, nb, ncol, dout, dcyc, grid);
            run<4>(d2, nb, ncol, dout, dcyc, grid);
            run<3>(d4, nb, ncol, dout, dcyc, grid);
        }
    }
    CK(hipFree(d1));
    CK(hipFree(d2));
    CK(hipFree(d4));
    CK(hipFree(dout));
    CK(hipFree(dcyc));
    return 0;
}
