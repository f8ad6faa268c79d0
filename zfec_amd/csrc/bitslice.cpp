// bitslice.cpp -- source generator and hipRTC JIT cache of the bit-sliced
// GF(2^8) matrix-apply kernels (see bitslice.hpp).
//
// The kernel computes the same thing as matapply_* in kernels.hip -- for each
// stripe, out_i = sum_j C[i][j] * in_j over GF(2^8), the work of fec_encode
// (zfec/fec.c:487-505) and fec_decode (zfec/fec.c:527-557) -- with the
// coefficient matrix compiled into the instruction stream.
//
// Per wave and unit: 2 KiB of each block (lane l owns bytes 16l..16l+15 and
// 1024+16l..1024+16l+15, so every load and store instruction is 1 KiB
// contiguous).  The 32 bytes of a lane are transposed into 8 bit-planes
// (plane a = bit a of all 32 bytes); an output plane b of c*x is the XOR of the
// input planes a with bit b of c*2^a set.  Rows are processed in register
// tiles of up to kBsMaxTile outputs (8 accumulator planes each); inside a tile
// every input is loaded, transposed, expanded into the XOR combinations of its
// planes 0-3 (L[1..15]) and 4-7 (H[1..15]), and each accumulator plane takes
// one XOR3 (acc ^ L[lo] ^ H[hi]).  The accumulators are transposed back to
// bytes and stored with streaming stores.
#include "bitslice.hpp"

#include <dirent.h>
#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <hip/hiprtc.h>

#include "config.hpp"
#include "gf256.hpp"

namespace zfec_hip {
namespace {

// masks[b]: bit a is set iff bit b of c*x depends on bit a of x, i.e. iff bit
// b of c * 2^a (2 = alpha, zfec/fec.c:16) is set.
void coef_masks(uint8_t c, uint8_t masks[8]) {
    const Field& f = field();
    for (int b = 0; b < 8; ++b) {
        unsigned m = 0;
        for (int a = 0; a < 8; ++a)
            if ((f.mul[c][1u << a] >> b) & 1u) m |= 1u << a;
        masks[b] = static_cast<uint8_t>(m);
    }
}

struct Src {
    std::string s;
    void operator()(const char* fmt, ...) __attribute__((format(printf, 2, 3))) {
        char buf[1024];
        va_list ap;
        va_start(ap, fmt);
        const int n = vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        if (n > 0) s.append(buf, static_cast<size_t>(n) < sizeof buf ? static_cast<size_t>(n) : sizeof buf - 1);
    }
};

const char* const kPrelude = R"PRE(typedef unsigned int u32;
typedef unsigned long long u64;
typedef unsigned char u8;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
// v_bitop3_b32 truth tables index the operands as S0 = 0xF0, S1 = 0xCC, S2 = 0xAA
__device__ __forceinline__ u32 x3(u32 a, u32 b, u32 c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ u32 sel(u32 m, u32 a, u32 b) { return __builtin_amdgcn_bitop3_b32(a, b, m, 0xE4); }  // m ? a : b
// one block swap of an 8x8 bit-matrix transpose, four byte lanes at once:
// a <- (a & m) | ((b << s) & ~m),  b <- ((a >> s) & m) | (b & ~m)
__device__ __forceinline__ void sw(u32& a, u32& b, int s, u32 m) {
    const u32 t0 = sel(m, a, b << s);
    const u32 t1 = sel(m, a >> s, b);
    a = t0;
    b = t1;
}
// Two block swaps with the same shift at once: the shifts as 64-bit register
// pairs (v_lshlrev_b64 / v_lshrrev_b64 shift two dwords at the issue rate of
// one 32-bit shift, tools/mb_valu.hip).  The bits that cross the dword
// boundary land exactly where the swap's mask discards them (the low s bits of
// a byte on the left shift, the high s bits on the right shift).  Inline asm,
// or the compiler splits the right shift back into v_alignbit + v_lshrrev.
// Pairs (a0, a1) and (b0, b1) are adjacent registers in the first two stages
// of tr8, where no moves are needed to form them.
__device__ __forceinline__ u64 shl64(u64 x, int s) {
    u64 r;
    asm("v_lshlrev_b64 %0, %1, %2" : "=v"(r) : "i"(s), "v"(x));
    return r;
}
__device__ __forceinline__ u64 shr64(u64 x, int s) {
    u64 r;
    asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "i"(s), "v"(x));
    return r;
}
__device__ __forceinline__ void sw2(u32& a0, u32& b0, u32& a1, u32& b1, int s, u32 m) {
    const u64 bl = shl64((((u64)b1) << 32) | b0, s);
    const u64 ar = shr64((((u64)a1) << 32) | a0, s);
    const u32 t0 = sel(m, a0, (u32)bl), t1 = sel(m, (u32)ar, b0);
    const u32 t2 = sel(m, a1, (u32)(bl >> 32)), t3 = sel(m, (u32)(ar >> 32), b1);
    a0 = t0;
    b0 = t1;
    a1 = t2;
    b1 = t3;
}
// 8 dwords (32 bytes) <-> 8 bit-planes; the transpose is its own inverse
__device__ __forceinline__ void tr8(u32& v0, u32& v1, u32& v2, u32& v3, u32& v4, u32& v5, u32& v6, u32& v7) {
#if ZFEC_SHIFT64
    sw2(v0, v4, v1, v5, 4, 0x0F0F0F0Fu); sw2(v2, v6, v3, v7, 4, 0x0F0F0F0Fu);
    sw2(v0, v2, v1, v3, 2, 0x33333333u); sw2(v4, v6, v5, v7, 2, 0x33333333u);
    sw(v0, v1, 1, 0x55555555u); sw(v2, v3, 1, 0x55555555u); sw(v4, v5, 1, 0x55555555u); sw(v6, v7, 1, 0x55555555u);
#else
    sw(v0, v4, 4, 0x0F0F0F0Fu); sw(v1, v5, 4, 0x0F0F0F0Fu); sw(v2, v6, 4, 0x0F0F0F0Fu); sw(v3, v7, 4, 0x0F0F0F0Fu);
    sw(v0, v2, 2, 0x33333333u); sw(v1, v3, 2, 0x33333333u); sw(v4, v6, 2, 0x33333333u); sw(v5, v7, 2, 0x33333333u);
    sw(v0, v1, 1, 0x55555555u); sw(v2, v3, 1, 0x55555555u); sw(v4, v5, 1, 0x55555555u); sw(v6, v7, 1, 0x55555555u);
#endif
}
// Buffer loads / stores off a wave-uniform base (block pointer + the unit's
// offset, in SGPRs) with the lane's 32-bit offset: no 64-bit VGPR address per
// block.  Store cache policy kStoreAux: 2 = nt (streaming), 16 = sc1,
// 17 = sc0 sc1, 18 = nt sc1.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(const u8* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<u8*>(p), (short)0, -1, 0x00020000);
}
__device__ __forceinline__ u32x4 ld(__amdgpu_buffer_rsrc_t r, u32 off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, u32 off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kStoreAux);
}
// LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes at p land at lds + 16 l
typedef __attribute__((address_space(1))) void GV;
typedef __attribute__((address_space(3))) void LV;
__device__ __forceinline__ void dma16(const u8* p, u32x4* lds) {
    __builtin_amdgcn_global_load_lds((const GV*)p, (LV*)lds, 16, 0, 0);
}
// the LDS-DMA writes have landed (hipcc orders no LDS read after them itself)
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
)PRE";

// Name of the XOR of input planes {base + a : bit a of m} of step n (m != 0),
// emitting the combinations it needs on first use.
struct Combos {
    unsigned n;
    char side;      // 'L' (planes 0-3) or 'H' (planes 4-7)
    unsigned base;  // 0 or 4
    bool have[16] = {};
    std::string name(unsigned m, Src& e) {
        char b[32];
        if ((m & (m - 1)) == 0) {  // one plane
            snprintf(b, sizeof b, "q%u_%u", n, base + static_cast<unsigned>(__builtin_ctz(m)));
            return b;
        }
        snprintf(b, sizeof b, "%c%u_%u", side, n, m);
        if (!have[m]) {
            const unsigned top = 1u << (31 - __builtin_clz(m));
            const std::string rest = name(m ^ top, e), one = name(top, e);
            e("    const u32 %s = %s ^ %s;\n", b, rest.c_str(), one.c_str());
            have[m] = true;
        }
        return b;
    }
};

}  // namespace

unsigned bitslice_tiles(unsigned r, const BsOptions& opt) {
    const unsigned maxt = opt.max_tile ? opt.max_tile : kBsMaxTile;
    return (r + maxt - 1) / maxt;
}

bool bitslice_split(unsigned r, const BsOptions& opt) {
    const unsigned nt = bitslice_tiles(r, opt);
    return opt.split && nt > 1 && nt <= 8;
}

bool bitslice_ksplit(unsigned k, unsigned r, const BsOptions& opt) {
    return opt.ksplit && k > 32 && bitslice_tiles(r, opt) == 1 && r <= 10;
}

namespace {
// The updates of one input step n (input j) to the accumulators of rows
// [r0, r1): acc ^= L[lo] ^ H[hi] per output plane (shared by both generators).
void emit_updates(Src& e, const std::vector<uint8_t>& masks, unsigned k, unsigned j, unsigned n, unsigned r0,
                  unsigned r1, std::vector<char>& init) {
    Combos lo{n, 'L', 0}, hi{n, 'H', 4};
    for (unsigned i = r0; i < r1; ++i) {
        const uint8_t* mk = &masks[(size_t(i) * k + j) * 8];
        for (unsigned b = 0; b < 8; ++b) {
            if (!mk[b]) continue;
            const unsigned ml = mk[b] & 15u, mh = unsigned(mk[b]) >> 4;
            const std::string sl = ml ? lo.name(ml, e) : std::string(), sh = mh ? hi.name(mh, e) : std::string();
            char acc[32];
            snprintf(acc, sizeof acc, "a%u_%u", i, b);
            char& ini = init[size_t(i - r0) * 8 + b];
            if (!ini) {
                if (ml && mh)
                    e("    %s = %s ^ %s;\n", acc, sl.c_str(), sh.c_str());
                else
                    e("    %s = %s;\n", acc, ml ? sl.c_str() : sh.c_str());
                ini = 1;
            } else if (ml && mh) {
                e("    %s = x3(%s, %s, %s);\n", acc, acc, sl.c_str(), sh.c_str());
            } else {
                e("    %s ^= %s;\n", acc, ml ? sl.c_str() : sh.c_str());
            }
        }
    }
}

// Wide codes with one row tile (k > 32, r <= 10; e.g. 94/100): the unit's
// inputs are split over the 4 waves of a workgroup (wave w: inputs
// [w*k/4, (w+1)*k/4)), each wave accumulates the partial planes of every row
// from its inputs, the partials go through LDS, and wave w reduces, transposes
// and stores rows w, w+4, ...  A 64 MiB stripe of 94/100 has 349 units of
// 2 KiB: one wave per unit leaves most of the chip idle, four per unit do not.
std::string source_ksplit(const std::vector<uint8_t>& masks, unsigned k, unsigned r, const BsOptions& opt,
                          const char* name) {
    Src e;
    e.s.reserve(size_t(r) * k * 8 * 40 + 8192);
    e("constexpr int kStoreAux = %u;\n#define ZFEC_SHIFT64 %d\n", 2u, 1);  // nt stores; 64-bit-shift transposes
    e.s += kPrelude;
    e("struct Args {\n  u64 sz, iss, oss;\n  u32 nstripes, cps, gs_c, gs_s;\n  const u8* in[%u];\n  u8* out[%u];\n};\n", k, r);
    e("extern \"C\" __global__ __launch_bounds__(256) void %s(const Args a) {\n", name);
    e("  const u32 lo16 = (threadIdx.x & 63u) * 16u;\n  const u32 lane = threadIdx.x & 63u;\n");
    e("  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n");
    const char* const PA = "ka->";
    e("  typedef __attribute__((address_space(4))) const Args* KArgs;\n"
          "  const KArgs ka0 = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();\n");
    auto launder = [&](const char* indent) {
        e("%sKArgs ka = ka0;\n%sasm volatile(\"\" : \"+s\"(ka));\n", indent, indent);
    };
    e("  __shared__ u32x4 red[%u];  // [row][wave][half][lane] partial planes\n", r * 4 * 2 * 64);
    e("  u32 s = blockIdx.x / a.cps, c = blockIdx.x - s * a.cps;\n");
    e("  while (s < a.nstripes) {\n");
    e("    u64 off = (u64)c * %uu;\n", kBsChunk);
    e("    if (off > a.sz - %uu) off = a.sz - %uu;  // the last chunk ends at sz (overlapping its neighbour)\n",
      kBsChunk, kBsChunk);
    e("    const u64 ub = (u64)s * a.iss + off, uo = (u64)s * a.oss + off;\n");
    for (unsigned i = 0; i < r; ++i)
        e("    u32 a%u_0, a%u_1, a%u_2, a%u_3, a%u_4, a%u_5, a%u_6, a%u_7;\n", i, i, i, i, i, i, i, i);
    const unsigned pf = opt.prefetch ? opt.prefetch : 1;
    for (unsigned w = 0; w < 4; ++w) {
        const unsigned j0 = w * k / 4, j1 = (w + 1) * k / 4;
        e("    if (wave == %uu) {  // inputs %u..%u\n", w, j0, j1 - 1);
        launder("    ");
        auto emit_load = [&](unsigned j) {
            e("    const __amdgpu_buffer_rsrc_t ri%u = rs(%sin[%u] + ub);\n", j, PA, j);
            e("    const u32x4 l%u_0 = ld(ri%u, lo16), l%u_1 = ld(ri%u, lo16 + 1024u);\n", j, j, j, j);
        };
        for (unsigned j = j0; j < j0 + pf && j < j1; ++j) emit_load(j);
        std::vector<char> init(size_t(r) * 8, 0);
        for (unsigned j = j0; j < j1; ++j) {
            if (j + pf < j1) emit_load(j + pf);
            e("    u32 q%u_0 = l%u_0.x, q%u_1 = l%u_0.y, q%u_2 = l%u_0.z, q%u_3 = l%u_0.w;\n", j, j, j, j, j, j, j, j);
            e("    u32 q%u_4 = l%u_1.x, q%u_5 = l%u_1.y, q%u_6 = l%u_1.z, q%u_7 = l%u_1.w;\n", j, j, j, j, j, j, j, j);
            e("    tr8(q%u_0, q%u_1, q%u_2, q%u_3, q%u_4, q%u_5, q%u_6, q%u_7);\n", j, j, j, j, j, j, j, j);
            emit_updates(e, masks, k, j, j, 0, r, init);
            e("    __builtin_amdgcn_sched_barrier(0);\n");
        }
        for (unsigned i = 0; i < r; ++i) {
            for (unsigned b = 0; b < 8; ++b)
                if (!init[size_t(i) * 8 + b]) e("    a%u_%u = 0u;\n", i, b);
            e("    red[%uu + lane] = u32x4{a%u_0, a%u_1, a%u_2, a%u_3};\n", (i * 4 + w) * 128, i, i, i, i);
            e("    red[%uu + lane] = u32x4{a%u_4, a%u_5, a%u_6, a%u_7};\n", (i * 4 + w) * 128 + 64, i, i, i, i);
        }
        e("    }\n");
    }
    e("    __syncthreads();\n");
    for (unsigned i = 0; i < r; ++i) {
        e("    if (wave == %uu) {  // row %u: the 4 partials\n", i % 4, i);
        launder("    ");
        e("    const u32x4 p%u_0 = red[%uu + lane] ^ red[%uu + lane] ^ red[%uu + lane] ^ red[%uu + lane];\n", i,
          (i * 4 + 0) * 128, (i * 4 + 1) * 128, (i * 4 + 2) * 128, (i * 4 + 3) * 128);
        e("    const u32x4 p%u_1 = red[%uu + lane] ^ red[%uu + lane] ^ red[%uu + lane] ^ red[%uu + lane];\n", i,
          (i * 4 + 0) * 128 + 64, (i * 4 + 1) * 128 + 64, (i * 4 + 2) * 128 + 64, (i * 4 + 3) * 128 + 64);
        e("    a%u_0 = p%u_0.x; a%u_1 = p%u_0.y; a%u_2 = p%u_0.z; a%u_3 = p%u_0.w;\n", i, i, i, i, i, i, i, i);
        e("    a%u_4 = p%u_1.x; a%u_5 = p%u_1.y; a%u_6 = p%u_1.z; a%u_7 = p%u_1.w;\n", i, i, i, i, i, i, i, i);
        e("    tr8(a%u_0, a%u_1, a%u_2, a%u_3, a%u_4, a%u_5, a%u_6, a%u_7);\n", i, i, i, i, i, i, i, i);
        e("    const __amdgpu_buffer_rsrc_t ro%u = rs(%sout[%u] + uo);\n", i, PA, i);
        e("    st(ro%u, lo16, u32x4{a%u_0, a%u_1, a%u_2, a%u_3});\n", i, i, i, i, i);
        e("    st(ro%u, lo16 + 1024u, u32x4{a%u_4, a%u_5, a%u_6, a%u_7});\n", i, i, i, i, i);
        e("    }\n");
    }
    e("    __syncthreads();  // every wave has read the partials before the next unit's overwrite\n");
    e("    c += a.gs_c;\n    s += a.gs_s;\n    if (c >= a.cps) { c -= a.cps; ++s; }\n  }\n}\n");
    return e.s;
}
}  // namespace

std::string bitslice_source(const uint8_t* coef, unsigned k, unsigned r, const BsOptions& opt, const char* name) {
    field_init();
    if (bitslice_ksplit(k, r, opt)) {
        std::vector<uint8_t> masks(size_t(r) * k * 8);
        for (unsigned i = 0; i < r; ++i)
            for (unsigned j = 0; j < k; ++j) coef_masks(coef[i * k + j], &masks[(size_t(i) * k + j) * 8]);
        return source_ksplit(masks, k, r, opt, name);
    }
    const unsigned ntiles = bitslice_tiles(r, opt);
    std::vector<unsigned> tile_lo(ntiles + 1);
    for (unsigned t = 0; t <= ntiles; ++t) tile_lo[t] = t * r / ntiles;  // near-equal tiles
    std::vector<uint8_t> masks(size_t(r) * k * 8);
    for (unsigned i = 0; i < r; ++i)
        for (unsigned j = 0; j < k; ++j) coef_masks(coef[i * k + j], &masks[(size_t(i) * k + j) * 8]);

    Src e;
    e.s.reserve(size_t(r) * k * 8 * 40 + 8192);
    e("constexpr int kStoreAux = %u;\n#define ZFEC_SHIFT64 %d\n", 2u, 1);  // nt stores; 64-bit-shift transposes
    e.s += kPrelude;
    e("struct Args {\n  u64 sz, iss, oss;\n  u32 nstripes, cps, gs_c, gs_s;\n  const u8* in[%u];\n  u8* out[%u];\n};\n", k, r);
    // split: the row tiles of a unit go to the waves of one workgroup, which
    // read the unit's inputs at the same time (L1/L2 hits instead of a re-read
    // from HBM per tile); otherwise each wave walks all tiles of its own unit.
    const bool split = bitslice_split(r, opt);
    const unsigned threads = split ? 64 * ntiles : 256;
    e("extern \"C\" __global__ __launch_bounds__(%u) void %s(const Args a) {\n", threads, name);
    e("  const u32 lo16 = (threadIdx.x & 63u) * 16u;\n");
    // argload: block pointers are read from the kernel-argument segment where
    // they are used, through a pointer the compiler must treat as new in every
    // scope (empty asm), instead of all being loaded up front and spilled
    const char* const PA = "ka->";
    e("  typedef __attribute__((address_space(4))) const Args* KArgs;\n"
          "  const KArgs ka0 = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();\n");
    auto launder = [&](const char* indent) {
        e("%sKArgs ka = ka0;\n%sasm volatile(\"\" : \"+s\"(ka));\n", indent, indent);
    };
    // share: the unit's inputs go through LDS in phases of `ph` (all k at once
    // when opt.phase is 0): a phase's inputs are loaded and transposed once,
    // by the waves in turn, then every wave applies them to its tile
    const unsigned ph = split && opt.share ? (opt.phase && opt.phase < k ? opt.phase : k) : 0;
    // dma: a phase's inputs go straight into LDS (LDS-DMA) and are transposed
    // in place; with more than one phase, two are resident and the next one
    // loads while the waves walk the current one (db)
    const bool db = split && opt.share && opt.dma && ph < k;
    const bool dma = db;
    if (split && opt.share) {
        e("  __shared__ u32x4 sh[%u];  // [buffer][input of the phase][half][lane] bit-planes\n", (db ? 2 : 1) * ph * 128);
        e("  const u32 lane = threadIdx.x & 63u;\n");
    }
    if (split) {
        e("  const u32 tile = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n");
        e("  const u32 wid = blockIdx.x;\n");
    } else {
        e("  const u32 wid = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n");
    }
    e("  u32 s = wid / a.cps, c = wid - s * a.cps;\n");
    e("  while (s < a.nstripes) {\n");
    e("    u64 off = (u64)c * %uu;\n", kBsChunk);
    e("    if (off > a.sz - %uu) off = a.sz - %uu;  // the last chunk ends at sz (overlapping its neighbour)\n",
      kBsChunk, kBsChunk);
    e("    const u64 ub = (u64)s * a.iss + off, uo = (u64)s * a.oss + off;\n");
    if (!split) launder("    ");

    // Steps: (tile t, input j) in order; loads run `prefetch` steps ahead
    // (across tiles, or inside each tile when split).
    const unsigned nsteps = ntiles * k;
    const unsigned pf = opt.prefetch;
    // share: each wave of the workgroup loads and transposes k / ntiles of the
    // unit's inputs once and leaves their bit-planes in LDS for all waves
    const bool share = split && opt.share;
    const char* const RS = "rs";
    auto emit_ld = [&](const char* ind, const char* dst, const char* rsrc, unsigned) {
        e("%sconst u32x4 %s_0 = ld(%s, lo16), %s_1 = ld(%s, lo16 + 1024u);\n", ind, dst, rsrc, dst, rsrc);
    };
    auto phase_base = [&](unsigned j) { return db ? (j / ph) % 2 * ph * 128 : 0u; };  // u32x4 offset of j's buffer
    auto emit_load = [&](unsigned n) {
        const unsigned j = n % k;
        if (share) {
            const unsigned sl = phase_base(j) + j % ph * 128;  // slot of input j in its phase's buffer
            e("    const u32x4 l%u_0 = sh[%uu + lane], l%u_1 = sh[%uu + lane];\n", n, sl, n, sl + 64);
            return;
        }
        char dst[16], rsrc[16];
        snprintf(dst, sizeof dst, "l%u", n);
        snprintf(rsrc, sizeof rsrc, "ri%u", n);
        e("    const __amdgpu_buffer_rsrc_t ri%u = %s(%sin[%u] + ub);\n", n, RS, PA, j);
        emit_ld("    ", dst, rsrc, j);
    };
    if (!split)
        for (unsigned n = 0; n < pf && n < nsteps; ++n) emit_load(n);
    // The load stage of phase [j0, j1) for the wave of tile t: inputs
    // j0 + t, j0 + t + ntiles, ... -> bit-planes -> LDS, then a barrier.  Every
    // tile branch runs the same phases, so the waves meet at the same barriers.
    // LDS-DMA of phase [j0, j1)'s inputs of the wave of tile t into its buffer,
    // and (after the wait) their in-place transposes
    auto emit_dma = [&](unsigned t, unsigned j0, unsigned j1) {
        e("    // inputs %u..%u -> LDS (DMA), one in %u per wave\n", j0, j1 - 1, ntiles);
        for (unsigned j = j0 + t; j < j1; j += ntiles) {
            const unsigned sl = phase_base(j) + (j - j0) * 128;
            e("    dma16(%sin[%u] + ub + lo16, sh + %uu);\n", PA, j, sl);
            e("    dma16(%sin[%u] + ub + lo16 + 1024u, sh + %uu);\n", PA, j, sl + 64);
        }
    };
    auto emit_xpose = [&](unsigned t, unsigned j0, unsigned j1) {
        e("    dma_wait();  // inputs %u..%u -> bit-planes in place\n", j0, j1 - 1);
        for (unsigned j = j0 + t; j < j1; j += ntiles) {
            const unsigned sl = phase_base(j) + (j - j0) * 128;
            e("    {\n      const u32x4 y0 = sh[%uu + lane], y1 = sh[%uu + lane];\n", sl, sl + 64);
            e("      u32 w0 = y0.x, w1 = y0.y, w2 = y0.z, w3 = y0.w, w4 = y1.x, w5 = y1.y, w6 = y1.z, w7 = y1.w;\n");
            e("      tr8(w0, w1, w2, w3, w4, w5, w6, w7);\n");
            e("      sh[%uu + lane] = u32x4{w0, w1, w2, w3};\n      sh[%uu + lane] = u32x4{w4, w5, w6, w7};\n    }\n", sl,
              sl + 64);
        }
    };
    auto emit_phase_load = [&](unsigned t, unsigned j0, unsigned j1) {
        if (dma) {
            emit_dma(t, j0, j1);
            emit_xpose(t, j0, j1);
            e("    __syncthreads();\n");
            return;
        }
        e("    // inputs %u..%u -> bit-planes -> LDS, one in %u per wave\n", j0, j1 - 1, ntiles);
        for (unsigned j = j0 + t; j < j1; j += ntiles) {
            char dst[16], rsrc[16];
            snprintf(dst, sizeof dst, "p%u", j);
            snprintf(rsrc, sizeof rsrc, "pi%u", j);
            e("    const __amdgpu_buffer_rsrc_t pi%u = %s(%sin[%u] + ub);\n", j, RS, PA, j);
            emit_ld("    ", dst, rsrc, j);
        }
        for (unsigned j = j0 + t; j < j1; j += ntiles) {
            e("    u32 w%u_0 = p%u_0.x, w%u_1 = p%u_0.y, w%u_2 = p%u_0.z, w%u_3 = p%u_0.w;\n", j, j, j, j, j, j, j, j);
            e("    u32 w%u_4 = p%u_1.x, w%u_5 = p%u_1.y, w%u_6 = p%u_1.z, w%u_7 = p%u_1.w;\n", j, j, j, j, j, j, j, j);
            e("    tr8(w%u_0, w%u_1, w%u_2, w%u_3, w%u_4, w%u_5, w%u_6, w%u_7);\n", j, j, j, j, j, j, j, j);
            e("    sh[%uu + lane] = u32x4{w%u_0, w%u_1, w%u_2, w%u_3};\n", (j - j0) * 128, j, j, j, j);
            e("    sh[%uu + lane] = u32x4{w%u_4, w%u_5, w%u_6, w%u_7};\n", (j - j0) * 128 + 64, j, j, j, j);
        }
        e("    __syncthreads();\n");
    };
    for (unsigned t = 0; t < ntiles; ++t) {
        const unsigned r0 = tile_lo[t], r1 = tile_lo[t + 1];
        const unsigned seq_end = split ? (t + 1) * k : nsteps;  // prefetch horizon
        e("    // tile %u: rows %u..%u\n", t, r0, r1 - 1);
        if (split) {
            e("    if (tile == %uu) {\n", t);
            launder("    ");
            if (!share)
                for (unsigned n = t * k; n < t * k + pf && n < seq_end; ++n) emit_load(n);
        }
        std::vector<char> init(size_t(r1 - r0) * 8, 0);
        for (unsigned i = r0; i < r1; ++i)
            e("    u32 a%u_0, a%u_1, a%u_2, a%u_3, a%u_4, a%u_5, a%u_6, a%u_7;\n", i, i, i, i, i, i, i, i);
        if (db) {  // the first phase's inputs (its barrier opens the phase loop)
            emit_dma(t, 0, ph);
            emit_xpose(t, 0, ph);
        }
        for (unsigned j = 0; j < k; ++j) {
            const unsigned n = t * k + j;
            if (share) {
                // LDS reads pf steps ahead inside the phase; the phase's load stage first
                const unsigned pe = (j / ph + 1) * ph < k ? (j / ph + 1) * ph : k;  // end of j's phase
                if (j % ph == 0 && db) {
                    // phase [j, pe)'s planes are in; every wave has walked the previous
                    // phase, whose buffer the next phase's DMA now overwrites
                    e("    __syncthreads();\n");
                    if (pe < k) emit_dma(t, pe, pe + ph < k ? pe + ph : k);
                    for (unsigned x = j; x < j + pf && x < pe; ++x) emit_load(t * k + x);
                } else if (j % ph == 0) {
                    if (j) e("    __syncthreads();  // the previous phase's planes are read\n");
                    emit_phase_load(t, j, pe);
                    for (unsigned x = j; x < j + pf && x < pe; ++x) emit_load(t * k + x);
                }
                if (pf == 0)
                    emit_load(n);
                else if (j + pf < pe)
                    emit_load(n + pf);
            } else if (pf == 0)
                emit_load(n);
            else if (n + pf < seq_end)
                emit_load(n + pf);
            e("    u32 q%u_0 = l%u_0.x, q%u_1 = l%u_0.y, q%u_2 = l%u_0.z, q%u_3 = l%u_0.w;\n", n, n, n, n, n, n, n, n);
            e("    u32 q%u_4 = l%u_1.x, q%u_5 = l%u_1.y, q%u_6 = l%u_1.z, q%u_7 = l%u_1.w;\n", n, n, n, n, n, n, n, n);
            if (!share)  // LDS holds planes already
                e("    tr8(q%u_0, q%u_1, q%u_2, q%u_3, q%u_4, q%u_5, q%u_6, q%u_7);\n", n, n, n, n, n, n, n, n);
            Combos lo{n, 'L', 0}, hi{n, 'H', 4};
            struct Upd {
                unsigned i, b, ml, mh;
            };
            std::vector<Upd> ups;
            for (unsigned i = r0; i < r1; ++i) {
                const uint8_t* mk = &masks[(size_t(i) * k + j) * 8];
                for (unsigned b = 0; b < 8; ++b)
                    if (mk[b]) ups.push_back(Upd{i, b, mk[b] & 15u, unsigned(mk[b]) >> 4});
            }
            auto update = [&](const Upd& u, const std::string& sl, const std::string& sh) {
                char acc[32];
                snprintf(acc, sizeof acc, "a%u_%u", u.i, u.b);
                char& ini = init[size_t(u.i - r0) * 8 + u.b];
                if (!ini) {
                    if (u.ml && u.mh)
                        e("    %s = %s ^ %s;\n", acc, sl.c_str(), sh.c_str());
                    else
                        e("    %s = %s;\n", acc, u.ml ? sl.c_str() : sh.c_str());
                    ini = 1;
                } else if (u.ml && u.mh) {
                    e("    %s = x3(%s, %s, %s);\n", acc, acc, sl.c_str(), sh.c_str());
                } else {
                    e("    %s ^= %s;\n", acc, u.ml ? sl.c_str() : sh.c_str());
                }
            };
            // combinations on first use, in row order
            for (const Upd& u : ups)
                update(u, u.ml ? lo.name(u.ml, e) : std::string(), u.mh ? hi.name(u.mh, e) : std::string());
            e("    __builtin_amdgcn_sched_barrier(0);\n");
            if (db && (j + 1) % ph == 0 && j + 1 < k)  // the last input of a phase: the next one's planes
                emit_xpose(t, j + 1, j + 1 + ph < k ? j + 1 + ph : k);
        }
        for (unsigned i = r0; i < r1; ++i) {
            for (unsigned b = 0; b < 8; ++b)
                if (!init[size_t(i - r0) * 8 + b]) e("    a%u_%u = 0u;\n", i, b);
            e("    tr8(a%u_0, a%u_1, a%u_2, a%u_3, a%u_4, a%u_5, a%u_6, a%u_7);\n", i, i, i, i, i, i, i, i);
            e("    const __amdgpu_buffer_rsrc_t ro%u = %s(%sout[%u] + uo);\n", i, RS, PA, i);
            e("    st(ro%u, lo16, u32x4{a%u_0, a%u_1, a%u_2, a%u_3});\n", i, i, i, i, i);
            e("    st(ro%u, lo16 + 1024u, u32x4{a%u_4, a%u_5, a%u_6, a%u_7});\n", i, i, i, i, i);
        }
        if (split) e("    }\n");
    }
    if (share) e("    __syncthreads();  // every wave has read the planes before the next unit's overwrite\n");
    e("    c += a.gs_c;\n    s += a.gs_s;\n    if (c >= a.cps) { c -= a.cps; ++s; }\n  }\n}\n");
    return e.s;
}

// ============================================================================
// hipRTC, disk cache, registry
// ============================================================================
namespace {

typedef hiprtcResult (*CreateFn)(hiprtcProgram*, const char*, const char*, int, const char**, const char**);
typedef hiprtcResult (*CompileFn)(hiprtcProgram, int, const char**);
typedef hiprtcResult (*SizeFn)(hiprtcProgram, size_t*);
typedef hiprtcResult (*GetFn)(hiprtcProgram, char*);
typedef hiprtcResult (*DestroyFn)(hiprtcProgram*);

struct Rtc {
    bool ok = false;
    std::string err;
    CreateFn create = nullptr;
    CompileFn compile = nullptr;
    SizeFn log_size = nullptr, code_size = nullptr;
    GetFn log = nullptr, code = nullptr;
    DestroyFn destroy = nullptr;
};

const Rtc& rtc() {
    static const Rtc r = [] {
        Rtc x;
        void* h = nullptr;
        for (const char* n : {"libhiprtc.so.7", "libhiprtc.so", "/opt/rocm/lib/libhiprtc.so.7", "/opt/rocm/lib/libhiprtc.so"})
            if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) {
            const char* d = dlerror();
            x.err = std::string("hipRTC not loadable: ") + (d ? d : "?");
            return x;
        }
        x.create = reinterpret_cast<CreateFn>(dlsym(h, "hiprtcCreateProgram"));
        x.compile = reinterpret_cast<CompileFn>(dlsym(h, "hiprtcCompileProgram"));
        x.log_size = reinterpret_cast<SizeFn>(dlsym(h, "hiprtcGetProgramLogSize"));
        x.log = reinterpret_cast<GetFn>(dlsym(h, "hiprtcGetProgramLog"));
        x.code_size = reinterpret_cast<SizeFn>(dlsym(h, "hiprtcGetCodeSize"));
        x.code = reinterpret_cast<GetFn>(dlsym(h, "hiprtcGetCode"));
        x.destroy = reinterpret_cast<DestroyFn>(dlsym(h, "hiprtcDestroyProgram"));
        x.ok = x.create && x.compile && x.log_size && x.log && x.code_size && x.code && x.destroy;
        if (!x.ok) x.err = "hipRTC symbols missing";
        return x;
    }();
    return r;
}

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
    for (unsigned char ch : s) {
        h ^= ch;
        h *= 1099511628211ull;
    }
    return h;
}

const char* const kRtcOptions[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-mcode-object-version=5"};
constexpr int kRtcNumOptions = sizeof(kRtcOptions) / sizeof(kRtcOptions[0]);

// Directory of the code-object cache: $ZFEC_HIP_JIT_CACHE ("" disables it),
// else jit_cache/ next to libzfec_hip.so (in-tree: compiled kernels travel
// with the build), if writable.
std::string cache_dir() {
    if (const char* e = getenv("ZFEC_HIP_JIT_CACHE")) return e;
    Dl_info info;
    if (!dladdr(reinterpret_cast<void*>(&cache_dir), &info) || !info.dli_fname) return std::string();
    std::string lib = info.dli_fname;
    const size_t slash = lib.rfind('/');
    const std::string d = (slash == std::string::npos ? std::string(".") : lib.substr(0, slash)) + "/jit_cache";
    mkdir(d.c_str(), 0755);
    return access(d.c_str(), W_OK | X_OK) == 0 ? d : std::string();
}

bool read_file(const std::string& path, std::vector<char>& out) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    std::vector<char> buf;
    char tmp[65536];
    size_t n;
    while ((n = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
    fclose(f);
    if (buf.size() < 64 || memcmp(buf.data(), "\x7f" "ELF", 4) != 0) return false;
    out.swap(buf);
    return true;
}

void write_file_atomic(const std::string& path, const std::vector<char>& data) {
    char suffix[64];
    snprintf(suffix, sizeof suffix, ".tmp.%d.%zx", static_cast<int>(getpid()),
             std::hash<std::thread::id>()(std::this_thread::get_id()));
    const std::string tmp = path + suffix;
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return;
    const bool ok = fwrite(data.data(), 1, data.size(), f) == data.size();
    if (fclose(f) == 0 && ok && rename(tmp.c_str(), path.c_str()) == 0) return;
    unlink(tmp.c_str());
}

// Code object for `src`: the disk cache, else hipRTC.
bool compile_code(const std::string& src, const std::string& name, std::vector<char>& code, std::string& err) {
    std::string opts;
    for (const char* o : kRtcOptions) (opts += o) += ' ';
    char hex[32];
    snprintf(hex, sizeof hex, "%016llx", static_cast<unsigned long long>(fnv1a(src, fnv1a(opts))));
    const std::string dir = cache_dir();
    const std::string path = dir.empty() ? std::string() : dir + "/" + name + "-" + hex + ".co";
    if (!path.empty() && read_file(path, code)) return true;
    if (const char* d = getenv("ZFEC_HIP_JIT_DUMP")) {  // the generated source, for offline inspection
        std::vector<char> text(src.begin(), src.end());
        write_file_atomic(std::string(d) + "/" + name + ".hip", text);
    }
    const Rtc& R = rtc();
    if (!R.ok) {
        err = R.err;
        return false;
    }
    hiprtcProgram prog;
    if (R.create(&prog, src.c_str(), (name + ".hip").c_str(), 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        err = "hiprtcCreateProgram failed";
        return false;
    }
    const char* opt_list[kRtcNumOptions];
    for (int i = 0; i < kRtcNumOptions; ++i) opt_list[i] = kRtcOptions[i];
    const hiprtcResult cr = R.compile(prog, kRtcNumOptions, opt_list);
    size_t n = 0;
    if (cr != HIPRTC_SUCCESS) {
        std::string log;
        if (R.log_size(prog, &n) == HIPRTC_SUCCESS && n > 1) {
            log.resize(n);
            R.log(prog, &log[0]);
        }
        err = "hipRTC compile of " + name + " failed: " + log.substr(0, 2000);
        R.destroy(&prog);
        return false;
    }
    if (R.code_size(prog, &n) != HIPRTC_SUCCESS || n == 0) {
        err = "hiprtcGetCodeSize failed";
        R.destroy(&prog);
        return false;
    }
    code.resize(n);
    R.code(prog, code.data());
    R.destroy(&prog);
    if (!path.empty()) write_file_atomic(path, code);
    return true;
}

struct Loaded {
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    int blocks_per_cu = 1;
    int num_cu = 256;
};

struct Entry {
    int state = 0;  // 0 compiling, 1 ready, 2 failed
    std::string name;
    unsigned threads = 256;          // workgroup size
    unsigned units_per_block = 4;    // units a workgroup covers per loop trip
    std::vector<char> code;
    std::map<int, Loaded> dev;
    int loading = -1;  // the device a prefetch worker is loading the module on
    unsigned k = 0, r = 0;
};

struct Registry {
    std::mutex mu;
    std::condition_variable cv;
    std::map<std::string, std::unique_ptr<Entry>> entries;
    std::map<std::string, int> seen;  // auto mode: launches of matrices not compiled yet
    int pending = 0, ready = 0;
    std::vector<std::thread> workers;
    std::string last_error;
    bool atexit_set = false;
};

Registry& reg() {
    static Registry* r = new Registry;  // never destroyed: compile threads may still run at exit
    return *r;
}

void join_workers() {
    Registry& R = reg();
    std::vector<std::thread> w;
    {
        std::lock_guard<std::mutex> g(R.mu);
        w.swap(R.workers);
    }
    for (auto& t : w)
        if (t.joinable()) t.join();
}

void run_compile(Entry* e, std::string src) {
    std::vector<char> code;
    std::string err;
    const bool ok = compile_code(src, e->name, code, err);
    Registry& R = reg();
    std::lock_guard<std::mutex> g(R.mu);
    if (ok) {
        e->code.swap(code);
        e->state = 1;
        ++R.ready;
    } else {
        e->state = 2;
        R.last_error = err;
        if (getenv("ZFEC_HIP_JIT_VERBOSE")) fprintf(stderr, "zfec_hip: %s\n", err.c_str());
    }
    --R.pending;
    R.cv.notify_all();
}

std::atomic<int> g_mode{-1};

// Options of a kernel for an r x k matrix: the configured ones, with the
// planes shared through LDS only while all k inputs' planes fit (2 KiB each),
// and, where all k at once would cap the residency below what the kernel's
// registers allow (~3 waves per SIMD, i.e. 12 / tiles workgroups per CU), in
// double-buffered LDS-DMA phases of 4 inputs: the r = 20 decode of K=20/M=60
// (2 tiles) 0.394 ms with register-loaded phases of 8 -> 0.377-0.382 (0.713 of
// HBM; phases of 2: 0.446).  Its r = 40 encode (4 tiles, register-bound)
// keeps one register-loaded phase of all 20 inputs: phases of 8 lost 0.678-0.691
// -> 0.665 of HBM, phases of 4 by DMA 0.600 -> 0.649 ms and one DMA phase
// 0.600 -> 0.615 (profiles/r05_jit_phase_ab.json, r05_lds_dma_ab.json).
// ZFEC_JIT_DMA_TILES_MAX (A/B knob, tools/ab_build.sh): the most row tiles a
// kernel may have and still take DMA phases.  3: 4-tile kernels (e.g. 30/70's
// r = 40 encode, 1024 x 1 MiB) keep one register-loaded phase of all k inputs,
// 0.600-0.603 ms with DMA phases of 4 against 0.586-0.588
// (profiles/r06_jit_dma_tiles_ab.json), as K=20/M=60's r = 40 encode does.
#ifndef ZFEC_JIT_DMA_TILES_MAX
#define ZFEC_JIT_DMA_TILES_MAX 3
#endif
BsOptions options_for(unsigned k, unsigned r) {
    BsOptions o;
    if (k > 32) o.share = false;
    const unsigned nt = bitslice_tiles(r, o);
    o.phase = k * 2u * 12u > 160u * nt && nt <= ZFEC_JIT_DMA_TILES_MAX ? 4u : 0u;
    o.dma = o.phase && o.phase < k;
    return o;
}

// Registry entry for (matrix, options); queues or runs its compile.  Called
// with R.mu held by `lk`; releases it while compiling synchronously.
std::string entry_key(const uint8_t* coef, unsigned k, unsigned r, const BsOptions& opt) {
    std::string key;
    key.reserve(64 + size_t(k) * r);
    char hdr[80];
    // (the layout of the earlier, configurable option set: kernel names, and
    // with them the code objects cached in jit_cache/, stay the same)
    snprintf(hdr, sizeof hdr, "%u/%u/%u/%u/1/2/0/0/%d/", k, r, opt.max_tile, opt.prefetch, opt.split ? 1 : 0);
    key += hdr;
    key += "argload/shift64/";
    if (opt.share && bitslice_split(r, opt)) {
        key += "share/";
        if (opt.phase && opt.phase < k) key += "phase" + std::to_string(opt.phase) + "/";
        if (opt.dma && opt.phase && opt.phase < k) key += "dma/";
    }
    if (bitslice_ksplit(k, r, opt)) key += "ksplit/";
    key.append(reinterpret_cast<const char*>(coef), size_t(k) * r);
    return key;
}

std::string kernel_name(const std::string& key, unsigned k, unsigned r) {
    char nm[80];
    snprintf(nm, sizeof nm, "zfec_hip_bitslice_k%u_r%u_%016llx", k, r, static_cast<unsigned long long>(fnv1a(key)));
    return nm;
}

// A new registry entry (state 0, one pending) for `key`.  R.mu held.
Entry* new_entry(const std::string& key, unsigned k, unsigned r, const BsOptions& opt) {
    Registry& R = reg();
    auto ne = std::make_unique<Entry>();
    Entry* e = ne.get();
    e->name = kernel_name(key, k, r);
    e->k = k;
    e->r = r;
    const bool ks = bitslice_ksplit(k, r, opt);
    e->threads = bitslice_split(r, opt) ? 64 * bitslice_tiles(r, opt) : 256;
    e->units_per_block = bitslice_split(r, opt) || ks ? 1 : 4;
    R.entries.emplace(key, std::move(ne));
    ++R.pending;
    return e;
}

// The module of a ready entry on device `dev` (the calling thread's current
// device): hipModuleLoadData (~7 ms for K=20/M=60's r = 40 kernel,
// tools/jit_load_probe.py), the function, its occupancy.
hipError_t load_module(const Entry& e, int dev, Loaded& nl) {
    hipError_t er = hipModuleLoadData(&nl.mod, e.code.data());
    if (er == hipSuccess) er = hipModuleGetFunction(&nl.fn, nl.mod, e.name.c_str());
    if (er != hipSuccess) {
        (void)hipGetLastError();
        return er;
    }
    int nb = 0;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, nl.fn, static_cast<int>(e.threads), 0) == hipSuccess &&
        nb > 0)
        nl.blocks_per_cu = nb;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0)
        nl.num_cu = ncu;
    return hipSuccess;
}

// One launch of a freshly loaded kernel with no work (nstripes = 0: every
// wave leaves its unit loop before touching memory) on a stream of its own:
// the runtime copies a module's code to the device at its first launch (~5 ms
// for K=20/M=60's r = 40 kernel, tools/jit_load_probe.py), which a prefetch
// must not leave to the caller's first launch.
bool warm_launch(const Entry& e, const Loaded& L) {
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    uint64_t args[5 + kMaxWideIn + kMaxOut] = {};  // sz, strides 0; nstripes 0, cps 1; null block pointers
    const uint32_t a32[4] = {0u, 1u, 0u, 1u};
    std::memcpy(&args[3], a32, sizeof a32);
    size_t size = (5 + e.k + e.r) * sizeof(uint64_t);  // struct Args of the generated source
    void* conf[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
    hipError_t er = hipModuleLaunchKernel(L.fn, 1, 1, 1, e.threads, 1, 1, 0, st, nullptr, conf);
    if (er == hipSuccess) er = hipStreamSynchronize(st);
    (void)hipStreamDestroy(st);
    if (er != hipSuccess) (void)hipGetLastError();
    return er == hipSuccess;
}

void spawn_worker(std::function<void()> f) {  // R.mu held
    Registry& R = reg();
    if (!R.atexit_set) {
        std::atexit(join_workers);
        R.atexit_set = true;
    }
    R.workers.emplace_back(std::move(f));
}

Entry* get_entry(const uint8_t* coef, unsigned k, unsigned r, bool sync, std::unique_lock<std::mutex>& lk) {
    Registry& R = reg();
    const BsOptions opt = options_for(k, r);
    const std::string key = entry_key(coef, k, r, opt);
    auto it = R.entries.find(key);
    if (it != R.entries.end()) return it->second.get();
    Entry* e = new_entry(key, k, r, opt);
    const char* nm = e->name.c_str();
    std::string src = bitslice_source(coef, k, r, opt, nm);
    if (sync) {
        lk.unlock();
        run_compile(e, std::move(src));
        lk.lock();
    } else {
        spawn_worker([e, s = std::move(src)]() mutable { run_compile(e, std::move(s)); });
    }
    return e;
}

// Names of the kernels whose code objects the disk cache holds (the part of a
// file name before "-<source hash>.co"), read once per process and cache
// directory: a code's construction (jit_prefetch) asks it, so it must cost a
// lookup.
bool on_disk(const std::string& name) {
    static std::mutex mu;
    static std::map<std::string, std::vector<std::string>> listed;
    const std::string dir = cache_dir();
    if (dir.empty()) return false;
    std::lock_guard<std::mutex> g(mu);
    auto it = listed.find(dir);
    if (it == listed.end()) {
        std::vector<std::string> v;
        if (DIR* d = opendir(dir.c_str())) {
            while (dirent* de = readdir(d)) {
                const std::string f = de->d_name;
                const size_t dash = f.rfind('-');
                if (dash != std::string::npos && f.size() > 3 && f.compare(f.size() - 3, 3, ".co") == 0)
                    v.push_back(f.substr(0, dash));
            }
            closedir(d);
        }
        it = listed.emplace(dir, std::move(v)).first;
    }
    return std::find(it->second.begin(), it->second.end(), name) != it->second.end();
}

// The other kernels serve the rest: few coefficients (memory-bound), blocks
// shorter than one unit, XOR-accumulating continuation passes, matrices past
// kJitMaxCoef, small launches (auto mode).
bool eligible(const ApplySpec& a, JitMode mode) {
    if (mode == kJitOff || a.accumulate || a.sz < static_cast<uint64_t>(kBsChunk) || a.nstripes == 0 || a.k == 0 ||
        a.r == 0 || a.k * a.r > kJitMaxCoef)
        return false;
    if (mode == kJitForce) return true;
    if (a.k * a.r < 24 || (a.k <= 4 && a.r <= 8)) return false;
    const double bytes = double(a.k + a.r) * double(a.sz) * double(a.nstripes);
    return bytes >= double(8u << 20);
}

// Auto mode compiles a matrix on its second eligible launch (a decode with a
// one-off erasure pattern does not queue a compile), and at most
// kAutoMaxKernels matrices in all.
constexpr int kAutoMinUses = 2;
constexpr size_t kAutoMaxKernels = 512;

// A thread's recent launches of ready kernels: the next launch of the same
// matrix on the same device (and configuration) skips the registry's lock,
// key string and map lookups.
struct Hit {
    const Config* cfg = nullptr;
    int dev = -1;
    unsigned k = 0, r = 0;
    std::vector<uint8_t> coef;
    Loaded L;
    const char* name = nullptr;
    unsigned threads = 0, upb = 0;
};
constexpr int kHits = 4;
thread_local Hit t_hits[kHits];
thread_local unsigned t_hit_next = 0;

}  // namespace

JitMode jit_mode() {
    int m = g_mode.load();
    if (m < 0) {
        const char* e = getenv("ZFEC_HIP_JIT");
        m = kJitAuto;
        if (e && (!strcmp(e, "0") || !strcmp(e, "off"))) m = kJitOff;
        if (e && (!strcmp(e, "2") || !strcmp(e, "force"))) m = kJitForce;
        int expect = -1;
        if (!g_mode.compare_exchange_strong(expect, m)) m = expect;  // set_jit_mode won the race
    }
    return static_cast<JitMode>(m);
}

void set_jit_mode(JitMode m) { g_mode.store(static_cast<int>(m)); }

int jit_prepare(const uint8_t* coef, unsigned k, unsigned r) {
    if (k == 0 || r == 0 || k * r > kJitMaxCoef) return -1;
    Registry& R = reg();
    std::unique_lock<std::mutex> lk(R.mu);
    Entry* e = get_entry(coef, k, r, true, lk);
    R.cv.wait(lk, [&] { return e->state != 0; });
    return e->state == 1 ? 0 : -1;
}

void jit_prefetch(const uint8_t* coef, unsigned k, unsigned r) {
    if (jit_mode() != kJitAuto || k == 0 || r == 0 || k * r > kJitMaxCoef || k * r < 24 || (k <= 4 && r <= 8)) return;
    const BsOptions opt = options_for(k, r);
    std::string key = entry_key(coef, k, r, opt);
    const std::string name = kernel_name(key, k, r);
    if (!on_disk(name)) return;  // never compiled here: no compile
    int dev = -1, ndev = 0;  // the caller's current device, whose module the worker loads
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        dev = -1;
    }
    Registry& R = reg();
    std::lock_guard<std::mutex> g(R.mu);
    if (R.entries.count(key) || R.entries.size() >= kAutoMaxKernels) return;
    Entry* e = new_entry(key, k, r, opt);
    // the source (its hash names the cached file) is generated by the worker:
    // ~10 ms at r = 40; then the module is loaded on `dev` (~7 ms), so the
    // first launch there finds the kernel ready
    e->loading = dev;  // until the worker is done, launches on dev keep to the other kernels
    ++R.pending;       // the module load: jit_wait waits for it too
    spawn_worker([e, m = std::vector<uint8_t>(coef, coef + size_t(k) * r), k, r, opt, dev]() {
        run_compile(e, bitslice_source(m.data(), k, r, opt, e->name.c_str()));
        Loaded nl;
        const bool ok = dev >= 0 && e->state == 1 && hipSetDevice(dev) == hipSuccess &&
                        load_module(*e, dev, nl) == hipSuccess && warm_launch(*e, nl);
        Registry& R = reg();
        std::lock_guard<std::mutex> g(R.mu);
        if (ok && !e->dev.count(dev)) e->dev.emplace(dev, nl);
        else if (ok) (void)hipModuleUnload(nl.mod);
        e->loading = -1;  // (a failed load: the launch path loads and reports)
        --R.pending;
        R.cv.notify_all();
    });
}

int jit_wait() {
    Registry& R = reg();
    std::unique_lock<std::mutex> lk(R.mu);
    R.cv.wait(lk, [&] { return R.pending == 0; });
    return R.ready;
}

std::string jit_last_error() {
    Registry& R = reg();
    std::lock_guard<std::mutex> g(R.mu);
    return R.last_error;
}

hipError_t launch_matapply_jit(const ApplySpec& a, hipStream_t stream, const char** name_out) {
    const JitMode mode = jit_mode();
    if (!eligible(a, mode)) return hipErrorNotSupported;
    const unsigned k = a.k, r = a.r;
    // the r x k matrix, contiguous
    uint8_t buf[kJitMaxCoef];
    const uint8_t* coef = a.coef;
    if (a.coef_stride != k) {
        for (unsigned i = 0; i < r; ++i) std::memcpy(buf + size_t(i) * k, a.coef + size_t(i) * a.coef_stride, k);
        coef = buf;
    }
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorNotSupported;
    const Config* cfg = &config();
    const Hit* hit = nullptr;
    for (const Hit& h : t_hits)
        if (h.name && h.cfg == cfg && h.dev == dev && h.k == k && h.r == r && !memcmp(h.coef.data(), coef, size_t(k) * r)) {
            hit = &h;
            break;
        }
    Loaded L;
    const char* name;
    unsigned threads, upb;
    if (hit) {
        L = hit->L;
        name = hit->name;
        threads = hit->threads;
        upb = hit->upb;
    } else {
        Registry& R = reg();
        std::unique_lock<std::mutex> lk(R.mu);
        if (mode == kJitAuto) {
            const std::string key = entry_key(coef, k, r, options_for(k, r));
            if (!R.entries.count(key)) {
                if (R.entries.size() >= kAutoMaxKernels) return hipErrorNotSupported;
                if (R.seen.size() > 4 * kAutoMaxKernels) R.seen.clear();
                if (++R.seen[key] < kAutoMinUses) return hipErrorNotSupported;
                R.seen.erase(key);
            }
        }
        Entry* e = get_entry(coef, k, r, mode == kJitForce, lk);
        if (e->state == 0) {
            if (mode != kJitForce) return hipErrorNotReady;
            R.cv.wait(lk, [&] { return e->state != 0; });
        }
        if (e->state != 1) return hipErrorNotSupported;
        auto it = e->dev.find(dev);
        if (it == e->dev.end() && e->loading == dev && mode != kJitForce)
            return hipErrorNotReady;  // a prefetch is loading it: no 7 ms load in a launch
        if (it == e->dev.end()) {
            Loaded nl;
            const hipError_t er = load_module(*e, dev, nl);
            if (er != hipSuccess) {
                e->state = 2;
                R.last_error = std::string("loading ") + e->name + ": " + hipGetErrorString(er);
                return hipErrorNotSupported;
            }
            it = e->dev.emplace(dev, nl).first;
        }
        L = it->second;
        name = e->name.c_str();  // stable: entries are never removed
        threads = e->threads;
        upb = e->units_per_block;
        lk.unlock();
        Hit& h = t_hits[t_hit_next++ % kHits];
        h.cfg = cfg;
        h.dev = dev;
        h.k = k;
        h.r = r;
        h.coef.assign(coef, coef + size_t(k) * r);
        h.L = L;
        h.name = name;
        h.threads = threads;
        h.upb = upb;
    }

    const uint64_t cps = (a.sz + kBsChunk - 1) / kBsChunk;
    const uint64_t waves = cps * a.nstripes;
    if (waves >= (1ull << 32) - (1ull << 24)) return hipErrorNotSupported;
    const uint64_t need = (waves + upb - 1) / upb;
    const uint64_t cap = uint64_t(L.num_cu) * L.blocks_per_cu * 64;
    const uint32_t grid = static_cast<uint32_t>(need < cap ? need : cap);
    const uint64_t gwaves = uint64_t(grid) * upb;  // units per grid-stride step
    // struct Args of the generated source: 3 x u64, 4 x u32, k + r pointers
    uint64_t args[5 + kMaxWideIn + kMaxOut];
    args[0] = a.sz;
    args[1] = a.in_sstride;
    args[2] = a.out_sstride;
    const uint32_t a32[4] = {static_cast<uint32_t>(a.nstripes), static_cast<uint32_t>(cps),
                             static_cast<uint32_t>(gwaves % cps), static_cast<uint32_t>(gwaves / cps)};
    std::memcpy(&args[3], a32, sizeof a32);
    for (unsigned j = 0; j < k; ++j) args[5 + j] = reinterpret_cast<uint64_t>(a.in[j]);
    for (unsigned i = 0; i < r; ++i) args[5 + k + i] = reinterpret_cast<uint64_t>(a.out[i]);
    size_t size = (5 + k + r) * sizeof(uint64_t);
    void* conf[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
    const hipError_t er = hipModuleLaunchKernel(L.fn, grid, 1, 1, threads, 1, 1, 0, stream, nullptr, conf);
    if (er == hipSuccess && name_out) *name_out = name;
    return er;
}

}  // namespace zfec_hip
