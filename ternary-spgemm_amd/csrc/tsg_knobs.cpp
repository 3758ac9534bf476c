// tsg_knobs.cpp -- the environment knobs of the library (A/B studies and
// tests), each parsed strictly against the values it accepts.
//
// None of these changes a result: every accepted value yields code that is
// bit-exact (emulated on the CPU and run in the GPU suite).  Code variants
// with WRONG results (TSG_JIT_DIAG: no barrier, no DMA, no X reads, ... --
// timing studies only) exist only in the diagnostic build of the library
// (-DTSG_DIAG: lib/libternary_spgemm_diag.so, `make diag`); the product
// library refuses the variable at registration.  A set knob whose value is
// not accepted is an error at registration (tcsc_hip_create*) and in the host
// codegen entry points -- never silently reinterpreted.
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "tsg_internal.h"
#include "../../include/ternary_spgemm_test.h"

namespace tsg {

namespace {

// splits on ',' (empty fields kept)
std::vector<std::string> fields(const char *v)
{
    std::vector<std::string> out(1);
    for (const char *p = v; *p; p++) {
        if (*p == ',') out.emplace_back();
        else out.back() += *p;
    }
    return out;
}

bool parse_i64(const std::string &s, int64_t lo, int64_t hi, int base = 10)
{
    if (s.empty()) return false;
    errno = 0;
    char *end = nullptr;
    const long long x = std::strtoll(s.c_str(), &end, base);
    return errno == 0 && end && *end == '\0' && x >= lo && x <= hi;
}

bool one_of(const char *v, std::initializer_list<const char *> ok)
{
    for (const char *o : ok)
        if (std::strcmp(v, o) == 0) return true;
    return false;
}

bool int_in(const char *v, int64_t lo, int64_t hi) { return parse_i64(v, lo, hi); }

// TSG_JIT_DMA = "spread,m0k[,lag]": spread in [0, 1], m0k 0|1, lag 1|2
bool dma_ok(const char *v)
{
    const auto f = fields(v);
    if (f.size() < 2 || f.size() > 3) return false;
    char *end = nullptr;
    const double sp = std::strtod(f[0].c_str(), &end);
    if (f[0].empty() || !end || *end || !(sp >= 0.0 && sp <= 1.0)) return false;
    return parse_i64(f[1], 0, 1) && (f.size() == 2 || parse_i64(f[2], 1, 2));
}

// TSG_JIT_CP = "dma,touch": hex cache-policy bits, each a subset of sc0|nt|sc1
bool cp_ok(const char *v)
{
    const auto f = fields(v);
    if (f.size() != 2) return false;
    for (const auto &s : f) {
        if (!parse_i64(s, 0, 0xffffffffll, 16)) return false;
        if (std::strtoull(s.c_str(), nullptr, 16) & ~0x2030000ull) return false;
    }
    return true;
}

// TSG_JIT_TOUCH = "first,count" in 8-KiB units, first >= 1 (the dispatcher may
// move the touch base 8 KiB back, tsg_capi.cpp pick_tnear), count <= 4, inside
// the tail padding
bool touch_ok(const char *v)
{
    const auto f = fields(v);
    if (f.size() != 2 || !parse_i64(f[0], 1, 64) || !parse_i64(f[1], 0, 4)) return false;
    return (std::atoll(f[0].c_str()) + std::atoll(f[1].c_str())) * 8192ll <= (int64_t)kJitTailPadWords * 4;
}

// TSG_JIT_READS = "G,RA": read group size >= 1, read-ahead >= 0, G + RA <= the 24 X slots
bool reads_ok(const char *v)
{
    const auto f = fields(v);
    if (f.size() != 2 || !parse_i64(f[0], 1, kJitSlots) || !parse_i64(f[1], 0, kJitSlots)) return false;
    return std::atoi(f[0].c_str()) + std::atoi(f[1].c_str()) <= kJitSlots;
}

#ifdef TSG_DIAG
// TSG_JIT_DIAG (diagnostic build only): comma list of code variants
bool diag_ok(const char *v)
{
    for (const auto &s : fields(v))
        if (!one_of(s.c_str(), {"nobar", "nodma", "notouch", "nolgkm", "noreads", "novm", "samecode", "samewave",
                                "pairwave", "simdpair", "balance4", "balance1", "anti4"}))
            return false;
    return true;
}
#endif

struct Knob {
    const char *name;
    const char *accepts;
    bool (*ok)(const char *);
};

const Knob kKnobs[] = {
    {"TSG_KERNEL", "jit | rx", [](const char *v) { return one_of(v, {"jit", "rx"}); }},
    {"TSG_JIT_NW", "64 | 32 | 16 | 8", [](const char *v) { return one_of(v, {"64", "32", "16", "8"}); }},
    {"TSG_JIT_WAVES", "8 | 4", [](const char *v) { return one_of(v, {"8", "4"}); }},
    {"TSG_JIT_FAR", "0 | 1", [](const char *v) { return one_of(v, {"0", "1"}); }},
    {"TSG_JIT_XDIRECT", "0 | 1", [](const char *v) { return one_of(v, {"0", "1"}); }},
    {"TSG_JIT_HALF", "0 | 1", [](const char *v) { return one_of(v, {"0", "1"}); }},
    {"TSG_JIT_PAIR", "0 | 1", [](const char *v) { return one_of(v, {"0", "1"}); }},
    {"TSG_JIT_QBLOCK", "16 | 8", [](const char *v) { return one_of(v, {"16", "8"}); }},
    {"TSG_JIT_STAGGER", "0 | 1", [](const char *v) { return one_of(v, {"0", "1"}); }},
    {"TSG_JIT_PRIO", "0 | 1", [](const char *v) { return one_of(v, {"0", "1"}); }},
    {"TSG_JIT_ROWS64_MAXM", "0..65536", [](const char *v) { return int_in(v, 0, 65536); }},
    {"TSG_JIT_NOALIGN", "0 | 1", [](const char *v) { return one_of(v, {"0", "1"}); }},
    {"TSG_JIT_GN", "1..1024", [](const char *v) { return int_in(v, 1, 1024); }},
    {"TSG_JIT_GM", "1..1024", [](const char *v) { return int_in(v, 1, 1024); }},
    {"TSG_JIT_TMASK", "0..255", [](const char *v) { return int_in(v, 0, 255); }},
    {"TSG_JIT_DMA", "spread[0..1],m0k[0|1][,lag[1|2]]", dma_ok},
    {"TSG_JIT_CP", "dma,touch (hex, bits of 0x2030000)", cp_ok},
    {"TSG_JIT_TOUCH", "first,count (8-KiB units, first >= 1, count <= 4)", touch_ok},
    {"TSG_JIT_READS", "G,RA (G >= 1, G + RA <= 24)", reads_ok},
    {"TSG_JIT_TGROUP", "0 | 1 | 2", [](const char *v) { return one_of(v, {"0", "1", "2"}); }},
    {"TSG_JIT_XTOUCH", "0 | 1", [](const char *v) { return one_of(v, {"0", "1"}); }},
    {"TSG_JIT_TNEAR", "0 | 1", [](const char *v) { return one_of(v, {"0", "1"}); }},
    {"TSG_JIT_TGAP", "0..65536 (bytes)", [](const char *v) { return int_in(v, 0, 65536); }},
    {"TSG_JIT_TROLL", "0..8 (rolling code touches, 8-KiB windows ahead)", [](const char *v) { return int_in(v, 0, 8); }},
    {"TSG_JIT_MIX", "reads,dma (0|1 each)",
     [](const char *v) { return one_of(v, {"0,0", "0,1", "1,0", "1,1"}); }},
    {"TSG_JIT_DIR", "a directory", [](const char *v) { return *v != '\0'; }},
    {"TSG_ELL_PC", "0 | 1", [](const char *v) { return one_of(v, {"0", "1"}); }},
    {"TSG_ELL_MAXM", "0..1024", [](const char *v) { return int_in(v, 0, 1024); }},
    {"TSG_ELL_PC_MAXMN", "0..2^40", [](const char *v) { return int_in(v, 0, 1ll << 40); }},
    {"TSG_ELL_VARIANT", "0..4", [](const char *v) { return int_in(v, 0, kEllVariants - 1); }},
    {"TSG_ELL_LA", "1 | 2", [](const char *v) { return one_of(v, {"1", "2"}); }},
    {"TSG_ELL_LG", "2 | 4 | 8 | 16", [](const char *v) { return one_of(v, {"2", "4", "8", "16"}); }},
    {"TSG_ELL_PC_E", "16 | 32 | 64", [](const char *v) { return one_of(v, {"16", "32", "64"}); }},
    {"TSG_ELL_COPIES", "1 | 2", [](const char *v) { return one_of(v, {"1", "2"}); }},
    {"TSG_ELL_WPG", "4 | 8 | 16", [](const char *v) { return one_of(v, {"4", "8", "16"}); }},
    {"TSG_ELL_SCHED", "0 | 1", [](const char *v) { return one_of(v, {"0", "1"}); }},
#ifdef TSG_DIAG
    {"TSG_JIT_DIAG", "nobar,nodma,notouch,nolgkm,noreads,novm,samecode,samewave,pairwave,simdpair,balance4,balance1,anti4", diag_ok},
#endif
};

const Knob *find(const char *name)
{
    for (const Knob &k : kKnobs)
        if (std::strcmp(k.name, name) == 0) return &k;
    return nullptr;
}

}  // namespace

std::string knob_check()
{
#ifndef TSG_DIAG
    if (const char *d = std::getenv("TSG_JIT_DIAG"))
        return std::string("TSG_JIT_DIAG=") + d +
               " selects diagnostic code variants with WRONG results; they exist only in the diagnostic build "
               "(lib/libternary_spgemm_diag.so, `make diag`) -- unset it to use this library";
#endif
    for (const Knob &k : kKnobs) {
        const char *v = std::getenv(k.name);
        if (v && !k.ok(v)) return std::string(k.name) + "=" + v + ": expected " + k.accepts;
    }
    return "";
}

const char *knob_value(const char *name)
{
    const Knob *k = find(name);
    const char *v = k ? std::getenv(name) : nullptr;
    return v && k->ok(v) ? v : nullptr;
}

bool diag_build()
{
#ifdef TSG_DIAG
    return true;
#else
    return false;
#endif
}

}  // namespace tsg

extern "C" const char *tsg_knob_check(void)
{
    static thread_local std::string msg;
    msg = tsg::knob_check();
    return msg.c_str();
}
