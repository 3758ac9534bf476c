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
struct Emit {
    std::vector<uint32_t> &c;
    // keep 8-byte instructions 8-byte aligned (hand-asm placement rule)
    void align8()
    {
        if (c.size() & 1) c.push_back(0xbf800000u);  // s_nop 0
    }
    // v_pk_add_f32 v[d:d+1], v[d:d+1], v[x:x+1] [neg_lo:[0,1] neg_hi:[0,1]]  (VOP3P;
    // the two halves are rows 0 and 1 of the lane: two IEEE adds)
    void pk_add(uint32_t d, uint32_t x, bool neg)
    {
        align8();
        c.push_back(0xd3b24000u | d | (neg ? 0x200u : 0u));
        c.push_back((3u << 27) | ((256u + x) << 9) | (256u + d) | (neg ? (2u << 29) : 0u));
    }
    // ds_read_b64 v[d:d+1], v[a] offset:off
    void ds_read_b64(uint32_t d, uint32_t a, uint32_t off)
    {
        align8();
        c.push_back(0xd8ec0000u | off);
        c.push_back((d << 24) | a);
    }
    // global_load_lds_dwordx4 v[voff], s[84:85]   (LDS-DMA, destination M0)
    void glds_x4(uint32_t voff)
    {
        align8();
        c.push_back(0xddf48000u);
        c.push_back((84u << 16) | voff);
    }
    // global_load_dword v107, v114, s[88:89]   (code prefetch into L2)
    void code_touch()
    {
        align8();
        c.push_back(0xdc508000u);
        c.push_back((107u << 24) | (88u << 16) | 114u);
    }
    void m0_lit(uint32_t v) { align8(); c.push_back(0xbefc00ffu); c.push_back(v); }  // s_mov_b32 m0, v
    void save_m0() { c.push_back(0xbed6007cu); }      // s_mov_b32 s86, m0
    void restore_m0() { c.push_back(0xbefc0056u); }   // s_mov_b32 m0, s86
    void base_reset() { c.push_back(0xbed40150u); }   // s_mov_b64 s[84:85], s[80:81]
    void base_next()                                  // s[84:85] += s82
    {
        c.push_back(0x80545254u);
        c.push_back(0x82558055u);
    }
    void touch_addr(uint32_t region_off)              // s[88:89] = s[92:93] + off
    {
        align8();
        c.push_back(0x8058ff5cu);
        c.push_back(region_off);
        c.push_back(0x8259805du);
    }
    void nop(uint32_t n = 0) { c.push_back(0xbf800000u | n); }
    void wait_lgkm0() { c.push_back(0xbf8cc07fu); }
    void wait_vm0() { c.push_back(0xbf8c0f70u); }
    void barrier() { c.push_back(0xbf8a0000u); }
    void ret() { c.push_back(0xbe801d5eu); }         // s_setpc_b64 s[94:95]
    uint32_t pos_bytes() const { return (uint32_t)(c.size() * 4); }
};

constexpr uint32_t kXSlot0 = 8;          // v[8 + 2s : 9 + 2s], s < kJitSlots
constexpr uint32_t kLdsBaseV = 104;      // v104 + b: lane row 0 of LDS buffer b
constexpr uint32_t kDmaOffV = 108;       // v108 + i: DMA piece i offsets
constexpr uint32_t kAcc0 = 116;          // column c: v[116 + 2c : 117 + 2c]
constexpr int kBlockRows = kJitSlots / 2;  // double-buffered X row blocks
constexpr uint32_t kRowBytes = kJitTileM * 4;             // one X^T row of the tile in LDS
constexpr uint32_t kBufBytes = kJitChunk * kRowBytes;     // one LDS chunk buffer
constexpr int kPieces = kJitChunk / kJitWaves / 2;        // DMA pieces per wave per chunk
constexpr uint32_t kTouchAhead = 8192;   // code prefetch window [pos + 8 KiB, pos + 24 KiB)
constexpr int kTailPad = 8192 + 1024;    // words of padding after the last stream (> 24 KiB)
static_assert(kJitChunk % (2 * kJitWaves) == 0, "chunk rows split in 2-row pieces over the waves");
static_assert(kPieces == 6, "register contract: v108-v113");
static_assert((kJitChunk - 1) * kRowBytes < 65536, "ds_read offset field");

// Rows of one step's chunk and their X slots.
struct Section {
    std::vector<int> rows;     // ascending chunk rows used by the wave's columns
    std::vector<int> slot;     // slot of rows[i]
    int nblk = 0;
};

}  // namespace

void build_jit_code(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin,
                    int K, int N, JitImage &img)
{
    img.K = K;
    img.N = N;
    img.Npad = ((N + kJitTileCols - 1) / kJitTileCols) * kJitTileCols;
    img.nch = std::max(1, (K + kJitChunk - 1) / kJitChunk);
    const int nch = img.nch, ntiles = img.Npad / kJitTileCols, steps = 2 * nch;
    img.wcode.assign((size_t)ntiles * kJitWaves, 0u);
    std::vector<uint32_t> &code = img.code;
    code.clear();
    const int64_t nnz = (int64_t)csp[N] + (int64_t)csn[N];
    code.reserve((size_t)nnz * 2 + (size_t)ntiles * kJitWaves * (steps * 220 + 64) + kTailPad + 64);
    code.insert(code.end(), {kJitMagic0, kJitMagic1, 0u, 0u});
    Emit E{code};

    std::vector<int32_t> cur((size_t)kJitNW * 2), end((size_t)kJitNW * 2);
    // rows of step q (chunk q % nch, pass q / nch) for the current pointers
    auto rows_of = [&](int q, Section &sec) {
        const int p = q / nch, klo = (q % nch) * kJitChunk, khi = klo + kJitChunk;
        const int32_t *ri = p ? rin : rip;
        bool used[kJitChunk] = {};
        for (int col = 0; col < kJitNW; col++) {
            const int32_t e = end[(size_t)col * 2 + p];
            for (int32_t i = cur[(size_t)col * 2 + p]; i < e && ri[i] < khi; i++) used[ri[i] - klo] = true;
        }
        sec.rows.clear();
        for (int r = 0; r < kJitChunk; r++)
            if (used[r]) sec.rows.push_back(r);
        sec.nblk = ((int)sec.rows.size() + kBlockRows - 1) / kBlockRows;
    };
    int gblk = 0;  // running block count of the stream: block parity = gblk & 1
    auto assign_slots = [&](Section &sec) {
        sec.slot.resize(sec.rows.size());
        for (size_t i = 0; i < sec.rows.size(); i++)
            sec.slot[i] = ((gblk + (int)(i / kBlockRows)) & 1) * kBlockRows + (int)(i % kBlockRows);
        gblk += sec.nblk;
    };
    auto emit_reads = [&](const Section &sec, int blk, int q) {
        const uint32_t vb = kLdsBaseV + (uint32_t)(q % 3);
        const size_t r0 = (size_t)blk * kBlockRows, r1 = std::min(sec.rows.size(), r0 + kBlockRows);
        for (size_t i = r0; i < r1; i++)
            E.ds_read_b64(kXSlot0 + 2u * (uint32_t)sec.slot[i], vb, (uint32_t)sec.rows[i] * kRowBytes);
    };
    int base_chunk = -1;  // chunk whose base s[84:85] holds
    auto emit_dma = [&](int q, int w) {  // stage step q's chunk into LDS buffer q % 3
        const int j = q % nch;
        if (j == 0) {
            E.base_reset();
        } else {
            if (base_chunk != j - 1) {  // not reached: chunks are staged in order
                E.base_reset();
                for (int i = 0; i < j; i++) E.base_next();
            } else {
                E.base_next();
            }
        }
        base_chunk = j;
        E.nop(4);  // SALU-written SGPR base -> VMEM
        for (int i = 0; i < kPieces; i++) {
            E.m0_lit((uint32_t)(q % 3) * kBufBytes + (uint32_t)(2 * (w * kPieces + i)) * kRowBytes);
            E.nop(0);  // M0 -> LDS-DMA
            E.glds_x4(kDmaOffV + (uint32_t)i);
        }
    };

    for (int t = 0; t < ntiles; t++) {
        for (int w = 0; w < kJitWaves; w++) {
            while (code.size() % 64) E.nop();  // 256-B aligned stream start
            img.wcode[(size_t)t * kJitWaves + w] = E.pos_bytes();
            const int n0 = t * kJitTileCols + w * kJitNW;
            for (int col = 0; col < kJitNW; col++)
                for (int p = 0; p < 2; p++) {
                    const int n = n0 + col;
                    const int32_t *cs = p ? csn : csp;
                    cur[(size_t)col * 2 + p] = n < N ? cs[n] : 0;
                    end[(size_t)col * 2 + p] = n < N ? cs[n + 1] : 0;
                }
            base_chunk = -1;
            gblk = 0;
            E.save_m0();
            // prologue: steps 0 and 1 staged, landed, visible
            emit_dma(0, w);
            emit_dma(1, w);
            E.wait_vm0();
            E.barrier();
            Section sec, next;
            bool prefetched = false;
            rows_of(0, sec);
            assign_slots(sec);
            for (int q = 0; q < steps; q++) {
                const int p = q / nch, klo = (q % nch) * kJitChunk;
                const bool neg = p == 1;
                const int32_t *ri = p ? rin : rip;
                if (q + 2 < steps) emit_dma(q + 2, w);
                for (uint32_t d = 0; d < 2; d++) {
                    E.touch_addr(E.pos_bytes() + kTouchAhead + d * 8192u);
                    E.nop(4);
                    E.code_touch();
                }
                if (sec.nblk > 0) {
                    if (!prefetched) emit_reads(sec, 0, q);
                    E.wait_lgkm0();
                }
                for (int blk = 0; blk < sec.nblk; blk++) {
                    if (blk + 1 < sec.nblk) emit_reads(sec, blk + 1, q);
                    const int rhi = (blk + 1 < sec.nblk) ? sec.rows[(size_t)(blk + 1) * kBlockRows] : kJitChunk;
                    // slot of a chunk row within this block
                    int slot_of[kJitChunk];
                    for (size_t i = (size_t)blk * kBlockRows; i < sec.rows.size() && sec.rows[i] < rhi; i++)
                        slot_of[sec.rows[i]] = sec.slot[i];
                    // columns in pairs, their entries interleaved (two independent
                    // chains back to back); each column keeps ascending k
                    for (int col = 0; col < kJitNW; col += 2) {
                        int32_t &ia = cur[(size_t)col * 2 + p], &ib = cur[(size_t)(col + 1) * 2 + p];
                        const int32_t ea = end[(size_t)col * 2 + p], eb = end[(size_t)(col + 1) * 2 + p];
                        const uint32_t acca = kAcc0 + 2u * (uint32_t)col, accb = acca + 2u;
                        for (;;) {
                            const bool ha = ia < ea && ri[ia] < klo + rhi, hb = ib < eb && ri[ib] < klo + rhi;
                            if (!ha && !hb) break;
                            if (ha) E.pk_add(acca, kXSlot0 + 2u * (uint32_t)slot_of[ri[ia++] - klo], neg);
                            if (hb) E.pk_add(accb, kXSlot0 + 2u * (uint32_t)slot_of[ri[ib++] - klo], neg);
                        }
                    }
                    if (blk + 1 < sec.nblk) E.wait_lgkm0();
                }
                // next step's first block: its chunk is already resident (staged
                // two steps ahead), so read it before the barrier
                prefetched = false;
                if (q + 1 < steps) {
                    rows_of(q + 1, next);
                    assign_slots(next);
                    if (next.nblk > 0) {
                        emit_reads(next, 0, q + 1);
                        prefetched = true;
                    }
                }
                E.wait_vm0();
                E.barrier();
                std::swap(sec, next);
            }
            E.restore_m0();
            E.ret();
        }
    }
    for (int i = 0; i < kTailPad; i++) E.nop();  // the code prefetch reads past the last stream
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
