// sparseGEMM_hip.cpp -- driver with the reference's command line and report
// format (cpp_impl/main.cpp:35-272), registering the MI355X kernel through the
// unchanged comp_func/add_function surface.  Its stdout can be scraped by the
// reference's run_benchmark.py regexes (run_benchmark.py:63-67):
//   "Running: <name>\n<cycles> cycles\nSpeedup is: <x>" (+ Performance /
//   Operational Intensity lines as with INSTRUMENTATION_RUN, main.cpp:264-271).
//
//   ./bin/sparseGEMM_hip.out -M 32 -K 1024 -N 4096 -s 4 [-correctness] [seed]
//
// Positional argv as the reference (main.cpp:49-57): M=argv[2], K=argv[4],
// N=argv[6], s=argv[8], "-correctness" at argv[9].  Inputs: the
// generateSparseMatrix law (tsg_gen_tcsc) and integer X in [-512,512]
// (tsg_gen_x), b = 2 (main.cpp:194), seeded (the reference seeds with time(0)).
#include <x86intrin.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tcsc_hip_plugin.hpp"

static std::vector<tsg::comp_func> userFuncs;  // main.cpp:12-14
static std::vector<std::string> funcNames;

static void add_function(tsg::comp_func f, std::string name)  // main.cpp:21-26
{
    userFuncs.push_back(f);
    funcNames.emplace_back(name);
}

struct HostTCSC {  // same public layout as class TCSC (TCSC.h:5-11)
    std::vector<int> col_start_pos, col_start_neg, row_index_pos, row_index_neg;
};

// Same public layout as BlockedTCSC<B> (BlockedTCSC.h:7-13), built from the
// TCSC: slot kb*N + n = column n's rows of block kb, K/B whole blocks.
template <int B>
struct HostBlockedTCSC {
    std::vector<int> col_start_pos, col_start_neg, row_index_pos, row_index_neg;
    HostBlockedTCSC(const HostTCSC &t, int K, int N)
    {
        for (int kb = 0; kb < K / B; kb++)
            for (int n = 0; n < N; n++) {
                col_start_pos.push_back((int)row_index_pos.size());
                col_start_neg.push_back((int)row_index_neg.size());
                for (int i = t.col_start_pos[n]; i < t.col_start_pos[n + 1]; i++)
                    if (t.row_index_pos[i] / B == kb) row_index_pos.push_back(t.row_index_pos[i]);
                for (int i = t.col_start_neg[n]; i < t.col_start_neg[n + 1]; i++)
                    if (t.row_index_neg[i] / B == kb) row_index_neg.push_back(t.row_index_neg[i]);
            }
        col_start_pos.push_back((int)row_index_pos.size());
        col_start_neg.push_back((int)row_index_neg.size());
    }
};
constexpr int kBlockSize = 512;  // BLOCK_SIZE, main.cpp:7

// Dense reference GEMM (the driver's own check, as sparseUtils.h:92-108 is the
// reference driver's): y = sum_k X[m,k]*W[k,n]; Y = y + b[n].
static void dense_gemm(const float *X, const int *W, const float *b, float *Y, int M, int N, int K)
{
#pragma omp parallel for schedule(static)
    for (int m = 0; m < M; m++)
        for (int n = 0; n < N; n++) {
            float y = 0.0f;
            for (int k = 0; k < K; k++) y += X[(size_t)m * K + k] * (float)W[(size_t)k * N + n];
            Y[(size_t)m * N + n] = y + b[n];
        }
}

// Cycle timing as perf.cpp:37-71: double the run count until >= 1e8 TSC
// cycles, then average.
static double rdtsc_time(const tsg::comp_func &f, float *X, float *B, float *Y, int M, int N, int K)
{
    int runs = 1;
    while (runs < (1 << 14)) {
        const unsigned long long t0 = __rdtsc();
        for (int i = 0; i < runs; i++) f(X, B, Y, M, N, K);
        if ((double)(__rdtsc() - t0) >= 1e8) break;
        runs *= 2;
    }
    const unsigned long long t0 = __rdtsc();
    for (int i = 0; i < runs; i++) f(X, B, Y, M, N, K);
    return (double)(__rdtsc() - t0) / runs;
}

int main(int argc, char **argv)
{
    std::printf("Starting program. ");
    if (argc < 9) {
        std::fprintf(stderr, "Usage: %s -M <int> -K <int> -N <int> -s <int> [-correctness] [seed]\n", argv[0]);
        return 1;
    }
    const int M = std::atoi(argv[2]), K = std::atoi(argv[4]), N = std::atoi(argv[6]);
    const int s = std::atoi(argv[8]);
    const bool correctness = argc > 9 && std::string(argv[9]) == "-correctness";
    const unsigned long long seed = argc > 10 ? std::strtoull(argv[10], nullptr, 10) : 42ull;

    HostTCSC W;
    int64_t np = 0, nn = 0;
    tsg::check(tsg_gen_tcsc(K, N, s, seed, 0, N, nullptr, nullptr, nullptr, nullptr, &np, &nn), "tsg_gen_tcsc");
    W.col_start_pos.resize(N + 1);
    W.col_start_neg.resize(N + 1);
    W.row_index_pos.resize(np > 0 ? np : 1);
    W.row_index_neg.resize(nn > 0 ? nn : 1);
    tsg::check(tsg_gen_tcsc(K, N, s, seed, 0, N, W.col_start_pos.data(), W.col_start_neg.data(),
                            W.row_index_pos.data(), W.row_index_neg.data(), &np, &nn),
               "tsg_gen_tcsc");
    W.row_index_pos.resize(np);
    W.row_index_neg.resize(nn);

    auto hw = std::make_shared<tsg::HipTCSC>(W, K, N);
    hw->reserve(M);  // compile the code image an M-row call runs before any timing
    add_function(tsg::make_hip_comp_func(hw), "HipBaseTCSC");
    // BaseBlockedTCSC over BlockedTCSC<512> (main.cpp:69,84-88), where K is a
    // whole number of blocks ("ASSUMING K DIVIDES B", BlockedTCSC.h:5)
    if (K >= kBlockSize && K % kBlockSize == 0)
        add_function(tsg::make_hip_comp_func(HostBlockedTCSC<kBlockSize>(W, K, N), K, N), "HipBaseBlockedTCSC");
    std::printf("%zu regular functions and 0 PrelU functions registered.\n", userFuncs.size());

    std::vector<float> X((size_t)M * K + 10), B(N, 2.0f), Y((size_t)M * N + 10, 0.0f);
    tsg::check(tsg_gen_x((int64_t)M * K, 512, seed + 1, X.data()), "tsg_gen_x");

    if (correctness) {
        std::vector<int> Wd = hw->getVectorRepresentation(K, N);
        std::vector<float> refY((size_t)M * N);
        dense_gemm(X.data(), Wd.data(), B.data(), refY.data(), M, N, K);
        for (size_t i = 0; i < userFuncs.size(); i++) {
            std::fill(Y.begin(), Y.end(), 0.0f);
            userFuncs[i](X.data(), B.data(), Y.data(), M, N, K);
            bool ok = true;
            for (size_t j = 0; j < (size_t)M * N && ok; j++)  // compare_results, tol 10e-6
                if (std::fabs(Y[j] - refY[j]) > 10e-6) {
                    std::printf("Error at: H=%zu, W=%zu, result=%g, groundTruth=%g\n", j / N, j % N, Y[j], refY[j]);
                    ok = false;
                }
            if (!ok) {
                std::printf("Test case \x1b[31m%s failed!\x1b[0m\n", funcNames[i].c_str());
                return 1;
            }
            std::printf("Test case %s passed!\n", funcNames[i].c_str());
        }
    }

    double base = 0;
    const double flops = (double)M * (double)(np + nn + N);  // comp.h:28-31,48-50,63
    const double bytes = 4.0 * ((double)M * K + (double)M * N + N) + 4.0 * (2.0 * (N + 1) + np + nn);
    for (size_t i = 0; i < userFuncs.size(); i++) {
        const double cyc = rdtsc_time(userFuncs[i], X.data(), B.data(), Y.data(), M, N, K);
        if (i == 0) base = cyc;
        std::printf("\nRunning: \x1b[31m%s\x1b[0m\n%g cycles\nSpeedup is: \x1b[32m%g\x1b[0m\n",
                    funcNames[i].c_str(), cyc, base / cyc);
        std::printf("Flops: %.0f\nPerformance: %g flops/cycle\nTotal Input Size: %.0f Bytes\n"
                    "Operational Intensity: %g Flops/Byte\nData Structure Size: %.0f Bytes\n",
                    flops, flops / cyc, bytes, flops / bytes, 4.0 * (2.0 * (N + 1) + np + nn));
    }
    return 0;
}
