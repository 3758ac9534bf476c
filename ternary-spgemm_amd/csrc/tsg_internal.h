// tsg_internal.h -- shared between the host planner, the C-ABI and the HIP
// kernels.  Not part of the public ABI (that is include/ternary_spgemm.h).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace tsg {

// Geometry of the LDS kernel (csrc/tcsc_kernels.hip).  The device image is
// built for exactly this geometry at registration.
constexpr int kLanes = 64;          // wavefront width (CDNA)
constexpr int kRowsPerLane = 2;     // M rows one lane accumulates (float2 = ds_read_b64)
constexpr int kTileM = kLanes * kRowsPerLane;  // 128 M rows per workgroup
constexpr int kChunkK = 128;        // K rows of X^T staged in LDS per chunk
constexpr int kZeroRow = kChunkK;   // LDS row holding +0.0f (pads index groups)
constexpr int kWaves = 4;           // waves per workgroup (256 threads)
constexpr int kEntPerWord = 4;      // uint8 row-in-chunk entries per dword

// Device image of one TCSC ("chunked TCSC"): for column n, pass p (0 = the
// +1 run, 1 = the -1 run) and K-chunk j, the entries of that column whose k
// lies in [j*kChunkK, (j+1)*kChunkK), in ascending k (the TCSC order), as
// uint8 (k - j*kChunkK), packed 4 per dword, the group padded with kZeroRow.
//   seg[((n*2 + p) * (nch+1)) + j]  = first dword of (n, p, j);
//   seg[... + j + 1]               = one past its last dword.
// Columns are padded to a multiple of the workgroup column tile with empty
// segments.  Entries for (n,p) are contiguous over j, so seg has nch+1 values.
struct Image {
    int K = 0, N = 0, Npad = 0, nch = 0;
    int tile_cols = 0;
    std::vector<uint32_t> seg;   // Npad * 2 * (nch + 1)
    std::vector<uint32_t> ent;   // packed entries (+ kEntTail dwords of padding)
};

// Builds the image from TCSC arrays (assumed validated).  tile_cols = N
// columns per workgroup; Npad = roundup(N, tile_cols).
void build_image(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                 const int32_t *rin, int K, int N, int tile_cols, Image &img);

std::string validate_tcsc(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                          const int32_t *rin, int K, int N);

// Kernel launchers (csrc/tcsc_kernels.hip).  All enqueue on `stream`.
// Mp/Kp: padded dims of the X^T work buffer (Mp % kTileM == 0, Kp = nch*kChunkK).
int launch_transpose(const float *X, float *XT, int M, int K, int Mp, int Kp, void *stream);
int launch_tcsc(const float *XT, int Mp, const uint32_t *seg, const uint32_t *ent,
                const float *b, const float *alpha, float *Y, int M, int N, int Npad,
                int nch, int tile_cols, int prelu, void *stream);

// Workgroup column tile used for an image (a function of N only).
int pick_tile_cols(int N);

}  // namespace tsg
