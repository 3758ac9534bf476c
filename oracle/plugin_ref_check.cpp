// plugin_ref_check.cpp -- the drop-in (include/tcsc_hip_plugin.hpp) compiled
// against the reference's OWN headers, read in place from /root/reference
// (never copied): cpp_impl/common.h (comp_func, comp_func_prelu, add_function,
// TCSC, BlockedTCSC, ...), data_structures/DataStructureInterface.hpp and
// sparseUtils.h (initX, generateSparseMatrix, GEMM, GEMM_PreLU,
// compare_results).  The plugin is built with TSG_WITH_REFERENCE_DSI, so
// tsg::HipTCSC really derives from the reference's DataStructureInterface
// (DataStructureInterface.hpp:4-14) and overrides its two pure virtuals.
//
// Registration is written exactly as INTEGRATION.md section 2 shows a
// maintainer adding it to cpp_impl/main.cpp:63-81, and the correctness loop
// is the reference's own (main.cpp:192-247): fresh Y, call, compare_results
// against the dense GEMM, "Test case <name> passed!" or exit(1).
//
// With `-perf` (after the reference's argv) the reference's benchmark loop
// follows (main.cpp:253-293): its own timing harness, cpp_impl/perf.cpp
// compiled UNMODIFIED with -DCALIBRATE (the x86 rdtsc path, perf.cpp:37-71,
// 298-339), times every registered comp_func -- "Running: / cycles / Speedup
// is:" relative to "BaseTCSC" (main.cpp:10,259-263).  "BaseTCSC" and
// "BaseTCSC_PreLU" are registered first, as main.cpp:76-81 registers them:
// comp.h does not build here (<arm_neon.h>, comp.h:6), so they are the
// oracle's restatements (oracle/tcsc_oracle.c, comp.h:25-69 and
// comp_prelu.h:12-70) -- test infrastructure, never in the package.
//
// TEST INFRASTRUCTURE: built by `make -C oracle refplugin` into
// oracle/_ref/plugin_ref_check (gitignored; travels to the GPU box like
// libref.so).  tests/test_integration_ref.py builds it on the CPU (compile +
// link = the ABI and the interface match); tests/test_gpu_parity.py runs it
// on the GPU when present.  Without a device it only reports that it linked.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "common.h"
#include "data_structures/DataStructureInterface.hpp"
#include "perf.h"
#include "sparseUtils.h"
#define TSG_WITH_REFERENCE_DSI
#include "tcsc_hip_plugin.hpp"

extern "C" {
#include "tcsc_oracle.h"
}

// the registry of main.cpp:12-33 (its definitions live in main.cpp, which has
// its own main(); the declarations come from common.h:15-16)
static std::vector<comp_func> userFuncs;
static std::vector<std::string> funcNames;
static std::vector<comp_func_prelu> userFuncs_prelu;
static std::vector<std::string> funcNames_prelu;

void add_function(comp_func f, std::string name)
{
    userFuncs.push_back(f);
    funcNames.push_back(name);
}

void add_prelu_function(comp_func_prelu f, std::string name)
{
    userFuncs_prelu.push_back(f);
    funcNames_prelu.push_back(name);
}

// threads for the reference GEMMs: OMP_NUM_THREADS (the GPU box's CPU share,
// 16) or the host's cores, at most 16 and one row block per thread at least
static unsigned ref_threads(int M)
{
    unsigned n = std::thread::hardware_concurrency();
    if (const char *e = std::getenv("OMP_NUM_THREADS")) n = (unsigned)std::max(1, std::atoi(e));
    return std::max(1u, std::min({n, 16u, (unsigned)std::max(M, 1)}));
}

int main(int argc, char **argv)
{
    // positional argv as main.cpp:49-52: -M m -K k -N n -s s
    int M = 96, K = 1536, N = 700, s = 4;
    if (argc >= 9) {
        M = std::atoi(argv[2]);
        K = std::atoi(argv[4]);
        N = std::atoi(argv[6]);
        s = std::atoi(argv[8]);
    }
    bool perf = false;
    for (int i = 1; i < argc; i++) perf = perf || std::strcmp(argv[i], "-perf") == 0;
    int ndev = 0;
    if (tcsc_hip_device_count(&ndev) != TSG_OK || ndev == 0) {
        std::printf("plugin_ref_check: built and linked against the reference headers; no HIP device, not run\n");
        return 0;
    }

    std::vector<int> W_raw = generateSparseMatrix<int>(K, N, s, false);  // main.cpp:60

    // the lines a maintainer adds to main.cpp
    auto sf_csc = std::make_shared<TCSC>(W_raw.data(), K, N);                            // main.cpp:63
    // "BaseTCSC" first, the speedup baseline (main.cpp:10,76-81): the oracle's
    // restatement of comp.h:25-69 over the reference ctor's arrays
    add_function([sf_csc](float *X, float *B, float *Y, int M, int N, int K) {
        oracle_base_tcsc(X, sf_csc->col_start_pos.data(), sf_csc->col_start_neg.data(),
                         sf_csc->row_index_pos.data(), sf_csc->row_index_neg.data(), B, Y, M, N, K);
    }, "BaseTCSC");
    add_prelu_function([sf_csc](float *X, float *B, float *alpha, float *Y, int M, int N, int K) {
        oracle_base_tcsc_prelu(X, sf_csc->col_start_pos.data(), sf_csc->col_start_neg.data(),
                               sf_csc->row_index_pos.data(), sf_csc->row_index_neg.data(), B, alpha, Y, M, N, K);
    }, "BaseTCSC_PreLU");
    add_function(tsg::make_hip_comp_func(*sf_csc, K, N), "HipBaseTCSC");
    auto sf_blocked = std::make_shared<BlockedTCSC<512>>(W_raw.data(), K, N);            // main.cpp:69
    add_function(tsg::make_hip_comp_func(*sf_blocked, K, N), "HipBaseBlockedTCSC");
    auto hip = std::make_shared<tsg::HipTCSC>(*sf_csc, K, N);
    add_prelu_function(tsg::make_hip_comp_func_prelu(hip), "HipBaseTCSC_PreLU");

    // DataStructureInterface (DataStructureInterface.hpp:10-13) through the base class
    std::unique_ptr<DataStructureInterface> dsi(new tsg::HipTCSC(W_raw.data(), K, N));
    const std::vector<int> back = dsi->getVectorRepresentation(K, N);
    if (back != W_raw) {
        std::printf("DataStructureInterface round trip failed\n");
        return 1;
    }
    std::printf("DataStructureInterface round trip passed!\n");

    // main.cpp:192-247
    std::vector<float> X_main = initX<float>(M * K, 512);
    std::vector<float> W_FP32_main(W_raw.begin(), W_raw.end());
    std::vector<float> B_main(N, 2);
    std::vector<float> alpha_main(N, 0.1);
    std::vector<float> Y_main(M * N, 0);
    std::vector<float> refY_main(M * N, 0);
    std::vector<float> refY_prelu_main(M * N, 0);
    // BlockedTCSC<512> drops rows past (K/512)*512 (BlockedTCSC.h:17): its reference is
    // the GEMM of that truncated W
    std::vector<float> W_blk(W_FP32_main);
    for (size_t i = (size_t)(K / 512) * 512 * N; i < W_blk.size(); i++) W_blk[i] = 0;
    std::vector<float> refY_blk(M * N, 0);
    // The reference's serial GEMM / GEMM_PreLU (sparseUtils.h:92-129), unchanged,
    // called on row blocks from several threads: every row of Y depends only on
    // its row of X, so the result is the one serial call's, bit for bit (at
    // configs[1] the three serial GEMMs take minutes on one core)
    const unsigned nt = ref_threads(M);
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nt; t++) {
        const int r0 = (int)((int64_t)M * t / nt), r1 = (int)((int64_t)M * (t + 1) / nt);
        if (r1 <= r0) continue;
        pool.emplace_back([&, r0, r1] {
            float *x = X_main.data() + (size_t)r0 * K;
            GEMM(x, W_FP32_main.data(), B_main.data(), refY_main.data() + (size_t)r0 * N, r1 - r0, N, K);
            GEMM_PreLU(x, W_FP32_main.data(), B_main.data(), alpha_main.data(), refY_prelu_main.data() + (size_t)r0 * N,
                       r1 - r0, N, K);
            GEMM(x, W_blk.data(), B_main.data(), refY_blk.data() + (size_t)r0 * N, r1 - r0, N, K);
        });
    }
    for (auto &th : pool) th.join();
    std::printf("reference GEMM / GEMM_PreLU done on %u thread(s) (M=%d K=%d N=%d s=%d)\n", nt, M, K, N, s);

    for (size_t i = 0; i < userFuncs.size(); i++) {
        std::fill(Y_main.begin(), Y_main.end(), 0);
        userFuncs[i](X_main.data(), B_main.data(), Y_main.data(), M, N, K);
        const std::vector<float> &ref = funcNames[i] == "HipBaseBlockedTCSC" ? refY_blk : refY_main;
        if (compare_results(Y_main.data(), const_cast<float *>(ref.data()), M, N)) {
            std::printf("Test case %s passed!\n", funcNames[i].c_str());
        } else {
            std::printf("Test case %s failed!\n", funcNames[i].c_str());
            return 1;
        }
    }
    for (size_t i = 0; i < userFuncs_prelu.size(); i++) {
        std::fill(Y_main.begin(), Y_main.end(), 0);
        userFuncs_prelu[i](X_main.data(), B_main.data(), alpha_main.data(), Y_main.data(), M, N, K);
        if (compare_results(Y_main.data(), refY_prelu_main.data(), M, N)) {
            std::printf("Test case %s passed!\n", funcNames_prelu[i].c_str());
        } else {
            std::printf("Test case %s failed!\n", funcNames_prelu[i].c_str());
            return 1;
        }
    }
    if (!perf) return 0;
    std::fflush(stdout);

    // main.cpp:253-293, the reference's benchmark loop around its perf_test
    // (perf.cpp, compiled unmodified): cycles per call, speedup vs BaseTCSC
    const int nonZero = s;  // main.cpp passes the sparsity argument as nonZero
    float base_cycles = 0;
    for (size_t i = 0; i < userFuncs.size(); i++) {
        const float perf_val = perf_test(userFuncs[i], M, K, N, nonZero);
        std::cout << "\nRunning: " << "\x1b[31m" << funcNames[i] << "\x1b[0m" << std::endl;
        std::cout << perf_val << " cycles" << std::endl;
        if (funcNames[i] == "BaseTCSC") base_cycles = perf_val;
        std::cout << "Speedup is: " << "\x1b[32m" << base_cycles / perf_val << "\x1b[0m" << std::endl;
    }
    float base_cycles_prelu = 0;
    for (size_t i = 0; i < userFuncs_prelu.size(); i++) {
        const float perf_val = perf_test_prelu(userFuncs_prelu[i], M, K, N, nonZero);
        std::cout << "\nRunning: " << "\x1b[31m" << funcNames_prelu[i] << "\x1b[0m" << std::endl;
        std::cout << perf_val << " cycles" << std::endl;
        if (funcNames_prelu[i] == "BaseTCSC_PreLU") base_cycles_prelu = perf_val;
        std::cout << "Speedup is: " << "\x1b[32m" << base_cycles_prelu / perf_val << "\x1b[0m" << std::endl;
    }
    return 0;
}
