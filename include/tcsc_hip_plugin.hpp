// tcsc_hip_plugin.hpp -- C++ adapter that plugs the C-ABI (ternary_spgemm.h)
// into the reference's registration surface unchanged:
//
//   using comp_func = std::function<void(float*X, float*B, float*Y, int M, int N, int K)>;
//   void add_function(comp_func f, std::string name);            // cpp_impl/common.h:12-15
//
//   auto sf_csc = std::make_shared<TCSC>(W_raw.data(), K, N);     // cpp_impl/main.cpp:63
//   add_function(tsg::make_hip_comp_func(*sf_csc, K, N), "HipBaseTCSC");
//
//   auto sf_blocked = std::make_shared<BlockedTCSC<BLOCK_SIZE>>(W_raw.data(), K, N);  // main.cpp:69
//   add_function(tsg::make_hip_comp_func(*sf_blocked, K, N), "HipBaseBlockedTCSC");
//   (BaseBlockedTCSC, comp.h:607-658; B deduced from BlockedTCSC<B>)
//
// HipTCSC also implements DataStructureInterface (init / getVectorRepresentation,
// cpp_impl/data_structures/DataStructureInterface.hpp:10-13); define
// TSG_WITH_REFERENCE_DSI after including the reference's header to inherit it.
//
// Error behaviour: the reference's comp_func returns void and failures surface
// through compare_results -> exit(1) (main.cpp:216-226).  Here every C-ABI
// failure throws std::runtime_error with tcsc_hip_last_error(): loud, never a
// silent CPU fallback.
#pragma once

#include <cstddef>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "ternary_spgemm.h"

namespace tsg {

using comp_func = std::function<void(float *X, float *B, float *Y, int M, int N, int K)>;
using comp_func_prelu =
    std::function<void(float *X, float *B, float *alpha, float *Y, int M, int N, int K)>;

inline void check(int rc, const char *where)
{
    if (rc != TSG_OK)
        throw std::runtime_error(std::string(where) + ": " + tcsc_hip_last_error());
}

class HipTCSC
#ifdef TSG_WITH_REFERENCE_DSI
    : public DataStructureInterface
#endif
{
public:
    HipTCSC() = default;
    HipTCSC(const int *matrix, int rows, int cols, int device = -1) : device_(device)
    {
        init(matrix, rows, cols);
    }
    // From any TCSC-shaped object with the reference's public vectors
    // (class TCSC, data_structures/TCSC.h:5-11).  Class types only: a raw
    // `int *` (main.cpp's W_raw.data()) is the dense-matrix ctor above.
    template <class TCSCLike, class = std::enable_if_t<std::is_class<TCSCLike>::value>>
    HipTCSC(const TCSCLike &t, int K, int N, int device = -1) : K_(K), N_(N), device_(device)
    {
        tsg_tcsc *h = nullptr;
        check(tcsc_hip_create(t.col_start_pos.data(), t.col_start_neg.data(),
                              t.row_index_pos.data(), t.row_index_neg.data(), K, N, device, &h),
              "tcsc_hip_create");
        h_.reset(h, tcsc_hip_destroy);
    }

    // From a BlockedTCSC<B>-shaped object (data_structures/BlockedTCSC.h:7-13):
    // calls compute BaseBlockedTCSC<float, B> (tcsc_hip_create_blocked).
    struct Blocked {};
    template <class BlockedLike>
    HipTCSC(Blocked, const BlockedLike &t, int K, int N, int B, int device = -1) : K_(K), N_(N), device_(device)
    {
        tsg_tcsc *h = nullptr;
        check(tcsc_hip_create_blocked(t.col_start_pos.data(), t.col_start_neg.data(), t.row_index_pos.data(),
                                      t.row_index_neg.data(), K, N, B, device, &h),
              "tcsc_hip_create_blocked");
        h_.reset(h, tcsc_hip_destroy);
    }

    // DataStructureInterface::init (DataStructureInterface.hpp:10)
    void init(const int *matrix, int rows, int cols)
#ifdef TSG_WITH_REFERENCE_DSI
        override
#endif
    {
        tsg_tcsc *h = nullptr;
        check(tcsc_hip_create_dense(matrix, rows, cols, device_, &h), "tcsc_hip_create_dense");
        h_.reset(h, tcsc_hip_destroy);
        K_ = rows;
        N_ = cols;
    }

    // DataStructureInterface::getVectorRepresentation (DataStructureInterface.hpp:13)
    std::vector<int> getVectorRepresentation(size_t rows, size_t cols)
#ifdef TSG_WITH_REFERENCE_DSI
        override
#endif
    {
        std::vector<int> W(rows * cols);
        check(tcsc_hip_to_dense(h_.get(), W.data(), (int)rows, (int)cols), "tcsc_hip_to_dense");
        return W;
    }

    // One comp_func call: host pointers, synchronous (BaseTCSC, comp.h:25-69).
    void operator()(float *X, float *B, float *Y, int M, int N, int K) const
    {
        check(tcsc_hip_gemm(h_.get(), X, B, Y, M, N, K), "tcsc_hip_gemm");
    }
    // comp_func_prelu (BaseTCSC_PreLU, comp_prelu.h:12-70).
    void prelu(float *X, float *B, float *alpha, float *Y, int M, int N, int K) const
    {
        check(tcsc_hip_gemm_prelu(h_.get(), X, B, alpha, Y, M, N, K), "tcsc_hip_gemm_prelu");
    }

    // Work buffer + the code image calls with up to max_M rows run, prepared
    // now (a first call would otherwise compile its stream width: tcsc_hip_reserve).
    void reserve(int max_M) const { check(tcsc_hip_reserve(h_.get(), max_M), "tcsc_hip_reserve"); }

    tsg_tcsc *handle() const { return h_.get(); }
    int K() const { return K_; }
    int N() const { return N_; }

private:
    std::shared_ptr<tsg_tcsc> h_;
    int K_ = 0, N_ = 0, device_ = -1;
};

// The registered lambda owns the device-resident format through a shared_ptr,
// as main.cpp:76-81 captures `sf_csc`.
inline comp_func make_hip_comp_func(std::shared_ptr<HipTCSC> w)
{
    return [w](float *X, float *B, float *Y, int M, int N, int K) { (*w)(X, B, Y, M, N, K); };
}
template <class TCSCLike>
comp_func make_hip_comp_func(const TCSCLike &t, int K, int N, int device = -1)
{
    return make_hip_comp_func(std::make_shared<HipTCSC>(t, K, N, device));
}
// BlockedTCSC<B> (any class template over the block size with the same public
// vectors): the more specialised overload, so the registration line reads as
// for TCSC.
template <template <int> class BlockedLike, int B>
comp_func make_hip_comp_func(const BlockedLike<B> &t, int K, int N, int device = -1)
{
    return make_hip_comp_func(std::make_shared<HipTCSC>(HipTCSC::Blocked{}, t, K, N, B, device));
}
inline comp_func_prelu make_hip_comp_func_prelu(std::shared_ptr<HipTCSC> w)
{
    return [w](float *X, float *B, float *alpha, float *Y, int M, int N, int K) {
        w->prelu(X, B, alpha, Y, M, N, K);
    };
}

}  // namespace tsg
