// tsg_jit.cpp -- host side of the weight-compiled ("jit") TCSC kernel:
//   1. build_jit_code: turns the TCSC arrays into gfx950 machine code, one
//      straight-line stream per (column tile, wave) (register contract:
//      tsg_jit_kernel.hip header);
//   2. JitModule::load: appends that code to the dispatcher's code object
//      (lib/tsg_jit.co) as a PT_LOAD R|X segment, patches the dispatcher's
//      region-base literal, and loads the image with hipModuleLoadData.
//
// Order contract (cpp_impl/comp.h:37-63, BaseTCSC): for every column the
// generated adds are its +1 entries in ascending k over all chunks, then its
// -1 entries in ascending k, one v_pk_add_f32 pair per entry (two IEEE adds,
// rows 0-1 and 2-3 of the lane); the dispatcher adds b[n] last.
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <elf.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <iterator>

#include "tsg_internal.h"
#include "../../include/ternary_spgemm.h"

namespace tsg {

namespace {

// --- gfx950 encodings (checked against llvm-mc -mcpu=gfx950 -show-encoding) ---
// v_pk_add_f32 v[d:d+1], v[d:d+1], v[x:x+1] [neg_lo:[0,1] neg_hi:[0,1]]  (VOP3P)
inline void emit_pk_add(std::vector<uint32_t> &c, uint32_t d, uint32_t x, bool neg)
{
    c.push_back(0xd3b24000u | d | (neg ? 0x200u : 0u));
    c.push_back((3u << 27) | ((256u + x) << 9) | (256u + d) | (neg ? (2u << 29) : 0u));
}
// ds_read_b128 v[d:d+3], v[a] offset:off  (DS)
inline void emit_ds_read_b128(std::vector<uint32_t> &c, uint32_t d, uint32_t a, uint32_t off)
{
    c.push_back(0xd9fe0000u | off);
    c.push_back((d << 24) | a);
}
inline void emit_wait_lgkm0(std::vector<uint32_t> &c) { c.push_back(0xbf8cc07fu); }
inline void emit_nop(std::vector<uint32_t> &c) { c.push_back(0xbf800000u); }
// s_getpc_b64 s[92:93]; s_setpc_b64 s[94:95]
inline void emit_return(std::vector<uint32_t> &c)
{
    c.push_back(0xbedc1c00u);
    c.push_back(0xbe801d5eu);
}

constexpr uint32_t kXSlot0 = 8;     // v[8 + 4s : 11 + 4s], s < kJitSlots
constexpr uint32_t kLdsBase0 = 104, kLdsBase1 = 105;
constexpr uint32_t kAcc0 = 112;     // column c: v[112 + 4c : 115 + 4c]
constexpr int kBlockRows = kJitSlots / 2;  // double-buffered X row blocks

}  // namespace

void build_jit_code(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin,
                    int K, int N, JitImage &img)
{
    img.K = K;
    img.N = N;
    img.Npad = ((N + kJitTileCols - 1) / kJitTileCols) * kJitTileCols;
    img.nch = std::max(1, (K + kJitChunk - 1) / kJitChunk);
    const int nch = img.nch, ntiles = img.Npad / kJitTileCols;
    img.wcode.assign((size_t)ntiles * kJitWaves, 0u);
    std::vector<uint32_t> &c = img.code;
    c.clear();
    const int64_t nnz = (int64_t)csp[N] + (int64_t)csn[N];
    c.reserve((size_t)nnz * 4 + (size_t)ntiles * kJitWaves * 2 * nch * 64 + 64);
    c.insert(c.end(), {kJitMagic0, kJitMagic1, 0u, 0u});

    std::vector<int32_t> cur((size_t)kJitNW * 2), end((size_t)kJitNW * 2);
    std::vector<int> slot_of(kJitChunk);
    std::vector<int> rows;
    for (int t = 0; t < ntiles; t++) {
        for (int w = 0; w < kJitWaves; w++) {
            while (c.size() % 64) emit_nop(c);  // 256-B aligned stream start
            img.wcode[(size_t)t * kJitWaves + w] = (uint32_t)(c.size() * 4);
            const int n0 = t * kJitTileCols + w * kJitNW;
            for (int col = 0; col < kJitNW; col++)
                for (int p = 0; p < 2; p++) {
                    const int n = n0 + col;
                    const int32_t *cs = p ? csn : csp;
                    cur[(size_t)col * 2 + p] = n < N ? cs[n] : 0;
                    end[(size_t)col * 2 + p] = n < N ? cs[n + 1] : 0;
                }
            for (int q = 0; q < 2 * nch; q++) {
                const int p = q / nch, j = q % nch;
                const bool neg = p == 1;
                const int32_t *ri = p ? rin : rip;
                const int klo = j * kJitChunk, khi = klo + kJitChunk;
                const uint32_t vb = (q & 1) ? kLdsBase1 : kLdsBase0;
                // rows of this chunk any of the wave's columns uses
                bool used[kJitChunk] = {};
                for (int col = 0; col < kJitNW; col++) {
                    const int32_t e = end[(size_t)col * 2 + p];
                    for (int32_t i = cur[(size_t)col * 2 + p]; i < e && ri[i] < khi; i++) used[ri[i] - klo] = true;
                }
                rows.clear();
                for (int r = 0; r < kJitChunk; r++)
                    if (used[r]) rows.push_back(r);
                const int nblk = ((int)rows.size() + kBlockRows - 1) / kBlockRows;
                for (size_t i = 0; i < rows.size(); i++)
                    slot_of[rows[i]] = (int)((i / kBlockRows) & 1) * kBlockRows + (int)(i % kBlockRows);
                auto emit_reads = [&](int blk) {
                    const size_t r0 = (size_t)blk * kBlockRows, r1 = std::min(rows.size(), r0 + kBlockRows);
                    for (size_t i = r0; i < r1; i++)
                        emit_ds_read_b128(c, kXSlot0 + 4u * (uint32_t)slot_of[rows[i]], vb,
                                          (uint32_t)rows[i] * 1024u);
                };
                if (nblk > 0) {
                    emit_reads(0);
                    emit_wait_lgkm0(c);
                    emit_nop(c);  // keeps the 8-byte VOP3P instructions 8-byte aligned
                }
                for (int blk = 0; blk < nblk; blk++) {
                    if (blk + 1 < nblk) emit_reads(blk + 1);
                    const int rhi = (blk + 1 < nblk) ? rows[(size_t)(blk + 1) * kBlockRows] : kJitChunk;
                    for (int col = 0; col < kJitNW; col++) {
                        int32_t &i = cur[(size_t)col * 2 + p];
                        const int32_t e = end[(size_t)col * 2 + p];
                        const uint32_t acc = kAcc0 + 4u * (uint32_t)col;
                        for (; i < e && ri[i] < klo + rhi; i++) {
                            const uint32_t x = kXSlot0 + 4u * (uint32_t)slot_of[ri[i] - klo];
                            emit_pk_add(c, acc, x, neg);
                            emit_pk_add(c, acc + 2, x + 2, neg);
                        }
                    }
                    if (blk + 1 < nblk) {
                        emit_wait_lgkm0(c);
                        emit_nop(c);
                    }
                }
                emit_return(c);
            }
        }
    }
}

// ------------------------------------------------------------ code object --
namespace {

std::string template_path()
{
    Dl_info info;
    if (dladdr(reinterpret_cast<void *>(&build_jit_code), &info) && info.dli_fname) {
        std::string p(info.dli_fname);
        const size_t s = p.rfind('/');
        return (s == std::string::npos ? std::string(".") : p.substr(0, s)) + "/tsg_jit.co";
    }
    return "tsg_jit.co";
}

}  // namespace

std::string JitModule::load(const std::vector<uint32_t> &code)
{
    const std::string path = template_path();
    std::ifstream f(path, std::ios::binary);
    if (!f) return "cannot open jit template " + path;
    std::vector<unsigned char> img((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (img.size() < sizeof(Elf64_Ehdr)) return "jit template too small";
    Elf64_Ehdr eh;
    std::memcpy(&eh, img.data(), sizeof eh);
    if (std::memcmp(eh.e_ident, ELFMAG, SELFMAG) != 0 || eh.e_ident[EI_CLASS] != ELFCLASS64 ||
        eh.e_phentsize != sizeof(Elf64_Phdr) || eh.e_phoff + (size_t)eh.e_phnum * sizeof(Elf64_Phdr) > img.size())
        return "jit template is not an ELF64 code object";
    // highest loaded address; the program header we turn into the code segment
    uint64_t top = 0;
    int spare = -1;
    for (int i = 0; i < eh.e_phnum; i++) {
        Elf64_Phdr ph;
        std::memcpy(&ph, img.data() + eh.e_phoff + (size_t)i * sizeof ph, sizeof ph);
        if (ph.p_type == PT_LOAD) top = std::max<uint64_t>(top, ph.p_vaddr + ph.p_memsz);
        if (ph.p_type == PT_GNU_STACK) spare = i;
    }
    if (spare < 0) return "jit template has no spare program header";
    const uint64_t page = 0x1000;
    const uint64_t vaddr = (top + page - 1) & ~(page - 1);
    // patch the dispatcher's literal: s_add_u32 s92, s92, 0x7a5e1234
    static const unsigned char pat[8] = {0x5c, 0xff, 0x5c, 0x80, 0x34, 0x12, 0x5e, 0x7a};
    size_t at = std::string::npos;
    for (size_t i = 0; i + 8 <= img.size(); i += 4)
        if (std::memcmp(img.data() + i, pat, 8) == 0) {
            if (at != std::string::npos) return "jit template: region literal not unique";
            at = i;
        }
    if (at == std::string::npos) return "jit template: region literal not found";
    uint64_t insn_vaddr = UINT64_MAX;
    for (int i = 0; i < eh.e_phnum; i++) {
        Elf64_Phdr ph;
        std::memcpy(&ph, img.data() + eh.e_phoff + (size_t)i * sizeof ph, sizeof ph);
        if (ph.p_type == PT_LOAD && at >= ph.p_offset && at < ph.p_offset + ph.p_filesz)
            insn_vaddr = ph.p_vaddr + (at - ph.p_offset);
    }
    if (insn_vaddr == UINT64_MAX || vaddr - insn_vaddr > 0xffffffffull) return "jit template: bad literal location";
    const uint32_t lit = (uint32_t)(vaddr - insn_vaddr);
    std::memcpy(img.data() + at + 4, &lit, 4);
    // append the code segment
    const size_t off = (img.size() + page - 1) & ~(size_t)(page - 1);
    const size_t bytes = code.size() * sizeof(uint32_t);
    img.resize(off + bytes, 0);
    std::memcpy(img.data() + off, code.data(), bytes);
    Elf64_Phdr ph = {};
    ph.p_type = PT_LOAD;
    ph.p_flags = PF_R | PF_X;
    ph.p_offset = off;
    ph.p_vaddr = ph.p_paddr = vaddr;
    ph.p_filesz = ph.p_memsz = bytes;
    ph.p_align = page;
    std::memcpy(img.data() + eh.e_phoff + (size_t)spare * sizeof ph, &ph, sizeof ph);

    hipModule_t m = nullptr;
    hipError_t e = hipModuleLoadData(&m, img.data());
    if (e != hipSuccess) return std::string("hipModuleLoadData: ") + hipGetErrorString(e);
    hipFunction_t fn = nullptr;
    e = hipModuleGetFunction(&fn, m, "tsg_jit_kernel");
    if (e != hipSuccess) {
        (void)hipModuleUnload(m);
        return std::string("hipModuleGetFunction: ") + hipGetErrorString(e);
    }
    module = m;
    function = fn;
    return "";
}

void JitModule::unload()
{
    if (module) (void)hipModuleUnload((hipModule_t)module);
    module = nullptr;
    function = nullptr;
}

int launch_tcsc_jit(const JitModule &jm, const float *XT, int Mp, const uint32_t *wcode, const float *b,
                    const float *alpha, float *Y, int M, int N, int Npad, int nch, int prelu,
                    uint32_t *status, void *stream)
{
    int mtiles = Mp / kJitTileM, ntiles = Npad / kJitTileCols;
    void *params[] = {(void *)&XT, (void *)&Mp, (void *)&wcode, (void *)&b, (void *)&alpha, (void *)&Y,
                      (void *)&M, (void *)&N, (void *)&nch, (void *)&mtiles, (void *)&ntiles, (void *)&prelu,
                      (void *)&status};
    hipError_t e = hipModuleLaunchKernel((hipFunction_t)jm.function, (unsigned)(mtiles * ntiles), 1, 1,
                                         kJitWaves * 64, 1, 1, 0, (hipStream_t)stream, params, nullptr);
    return e == hipSuccess ? 0 : -1;
}

}  // namespace tsg

// ---------------------------------------------------------------- C-ABI --
extern thread_local std::string g_tsg_host_err;

extern "C" int tsg_jit_codegen(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                               const int32_t *rin, int K, int N, uint32_t *code, int64_t code_cap,
                               int64_t *code_len, uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len)
{
    const std::string e = tsg::validate_tcsc(csp, csn, rip, rin, K, N);
    if (!e.empty()) {
        g_tsg_host_err = "tsg_jit_codegen: malformed TCSC: " + e;
        return TSG_ERR_ARG;
    }
    tsg::JitImage img;
    tsg::build_jit_code(csp, csn, rip, rin, K, N, img);
    if (code_len) *code_len = (int64_t)img.code.size();
    if (wcode_len) *wcode_len = (int64_t)img.wcode.size();
    if ((code && code_cap < (int64_t)img.code.size()) || (wcode && wcode_cap < (int64_t)img.wcode.size())) {
        g_tsg_host_err = "tsg_jit_codegen: buffer too small";
        return TSG_ERR_ARG;
    }
    if (code) std::memcpy(code, img.code.data(), img.code.size() * 4);
    if (wcode) std::memcpy(wcode, img.wcode.data(), img.wcode.size() * 4);
    return TSG_OK;
}
