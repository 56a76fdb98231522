// mh_common.h -- device code shared by the step kernels (mh_chain.hip: full evaluation,
// mh_delta.hip: incremental evaluation): the RNG, the reference's numerics for every cost term,
// the proposal draws and the accept rule. Everything here rounds exactly where
// KernelFolder/Kernel/Kernel.cu does (compile with -ffp-contract=off).
#pragma once

#include <hip/hip_runtime.h>
#include <rocrand/rocrand_philox4x32_10.h>
#include <rocrand/rocrand_uniform.h>

#include <stdint.h>

#include "mh_launch.h"
#include "mh_math.h"

#ifndef MH_ABLATE_OCML
#define MH_ABLATE_OCML 0  // timing-only builds: bit mask of the transcendentals taken from the
                          // device library (1 Box-Muller, 2 atan2, 4 cosf, 8 exp; results differ)
#endif
#ifndef MH_ABLATE
#define MH_ABLATE 0  // timing-only builds (tools/build_ablate.sh) compile phases out; product = 0
#endif

#ifndef MH_OPT
#define MH_OPT 0  // A/B switches of optimisations under measurement (bit per change)
#endif

#ifndef MH_CHECK
#define MH_CHECK 0  // debug builds: computed global / LDS indices validated and every decision of
                    // the rejection bound verified against the exact costs, the first violation
                    // recorded (mh_debug_check / mh_debug_check_delta); product = 0
#endif
#if MH_CHECK
static __device__ unsigned int g_check[8];  // (per translation unit) [0] violations, [1] site,
                                            // [2] [3] values, [4] wave, [5] checks made
static __device__ unsigned long long g_decide[4];  // steps that evaluated the bound, certain
                                                   // rejects, certain accepts, exact passes of
                                                   // the current configuration
__device__ __forceinline__ void mh_count_decision(int d, bool evaluated) {
    if (evaluated) atomicAdd(&g_decide[0], 1ull);
    if (d == 1) atomicAdd(&g_decide[1], 1ull);
    if (d == 2) atomicAdd(&g_decide[2], 1ull);
}
__device__ __forceinline__ bool mh_check_fail(unsigned site, unsigned v0, unsigned v1) {
    if (atomicAdd(&g_check[0], 1u) == 0u) {
        g_check[1] = site;
        g_check[2] = v0;
        g_check[3] = v1;
        g_check[4] = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    }
    return false;
}
#define MH_CK(ok, site, v0, v1) ((ok) ? true : mh_check_fail((site), (unsigned)(v0), (unsigned)(v1)))
#else
#define MH_CK(ok, site, v0, v1) (true)
#endif

namespace mh {

struct alignas(16) ObjP {  // per-object pose words read by the O(N^2) symmetry scan: one ds_read_b128
    float xf, yf;  // (float)x, (float)y -- every O(N^2) use of x, y is through float args
    float rotYf;   // (float)rotY
    float pad;
};

// 16-byte value loads. Memory is only ever accessed through its own type: a vector view of an
// ObjP or of a double / float stream is a byte copy into a local (one ds_read_b128 for 16-byte
// aligned LDS), never a dereference of a pointer cast to another object type, which strict
// aliasing lets the optimiser reorder against the real type's stores (tests/test_abi.py
// test_no_type_punning keeps it that way).
template <class V, class T>
__device__ __forceinline__ V load16(const T* p) {
    static_assert(sizeof(V) == 16, "16-byte loads only");
    V v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 16), 16);
    return v;
}
__device__ __forceinline__ float4 objp_f4(const ObjP& p) { return load16<float4>(&p); }

// ---- wave-level helpers -----------------------------------------------------------------

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- cross-lane LDS hand-offs -------------------------------------------------------------
// LDS that some lanes of a wavefront write and other lanes read changes hands in phases (round
// 3 lost chains to a missing wave_sync after a one-lane store). Lanes write through a Staged<T>
// view (put, or a record's fields through ->); a hand-off -- the only wave_sync outside this
// header -- makes the writes every lane's and orders every earlier read before later writes:
//  * publish(staged...) returns Published<T> views (reads only) of the arrays it is given, and
//    restage(published...) hands them back for rewriting: the speculative kernel's locals;
//  * the full-evaluation and incremental kernels keep their chain's arrays in ChainPtrs /
//    DeltaPtrs as Published<T> members, so a plain assignment to one does not compile: a lane
//    writes through stage(ch.X) and the phase ends in hand_off(ch.X, ...), which names the arrays
//    changing hands there.
template <class T>
struct Published {
    const T* p;
    __device__ __forceinline__ const T& operator[](int i) const { return p[i]; }
    __device__ __forceinline__ const T* ptr() const { return p; }
    __device__ __forceinline__ const T* operator->() const { return p; }
    __device__ __forceinline__ Published<T> at(int off) const { return Published<T>{p + off}; }
};
template <class T>
struct Staged {
    T* p;
    __device__ __forceinline__ void put(int i, const T& v) const { p[i] = v; }
    __device__ __forceinline__ Staged<T> at(int off) const { return Staged<T>{p + off}; }
    __device__ __forceinline__ T* operator->() const { return p; }  // (a record's fields)
    __device__ __forceinline__ T* ptr() const { return p; }
};
// This lane is about to write an array whose readers hold its Published view: its writes reach
// other lanes at the next hand_off() naming the array (no synchronisation here).
template <class T>
__device__ __forceinline__ Staged<T> stage(const Published<T>& v) {
    return Staged<T>{const_cast<T*>(v.p)};
}
// The hand-off of the arrays named: one wave_sync (the arguments document what changes hands).
template <class... T>
__device__ __forceinline__ void hand_off(const Published<T>&...) {
    wave_sync();
}
// publish(a, ...): one wave_sync, then the arrays' read views (`auto [av, bv] = publish(a, b);`).
template <class A, class B>
struct Pub2 { Published<A> a; Published<B> b; };
template <class A, class B, class C>
struct Pub3 { Published<A> a; Published<B> b; Published<C> c; };
template <class A>
__device__ __forceinline__ Published<A> publish(const Staged<A>& a) {
    wave_sync();
    return Published<A>{a.p};
}
template <class A, class B>
__device__ __forceinline__ Pub2<A, B> publish(const Staged<A>& a, const Staged<B>& b) {
    wave_sync();
    return Pub2<A, B>{{a.p}, {b.p}};
}
template <class A, class B, class C>
__device__ __forceinline__ Pub3<A, B, C> publish(const Staged<A>& a, const Staged<B>& b,
                                                 const Staged<C>& c) {
    wave_sync();
    return Pub3<A, B, C>{{a.p}, {b.p}, {c.p}};
}
// The same between the wavefronts of a workgroup (the workgroup barrier instead).
template <class A>
__device__ __forceinline__ Published<A> publish_workgroup(const Staged<A>& a) {
    __syncthreads();
    return Published<A>{a.p};
}
template <class A, class B, class C, class D>
struct Pub4 { Published<A> a; Published<B> b; Published<C> c; Published<D> d; };
template <class A, class B, class C, class D>
__device__ __forceinline__ Pub4<A, B, C, D> publish_workgroup(const Staged<A>& a, const Staged<B>& b,
                                                              const Staged<C>& c, const Staged<D>& d) {
    __syncthreads();
    return Pub4<A, B, C, D>{{a.p}, {b.p}, {c.p}, {d.p}};
}
// The receiving side of another wavefront's publish_workgroup(a, b, c, d): the same barrier,
// then the read views.
template <class A, class B, class C, class D>
__device__ __forceinline__ Pub4<A, B, C, D> receive_workgroup(const A* a, const B* b, const C* c,
                                                              const D* d) {
    __syncthreads();
    return Pub4<A, B, C, D>{{a}, {b}, {c}, {d}};
}
template <class T>
__device__ __forceinline__ Staged<T> restage(const Published<T>& v) {
    wave_sync();
    return Staged<T>{const_cast<T*>(v.p)};
}
template <class A, class B, class C>
struct Stg3 { Staged<A> a; Staged<B> b; Staged<C> c; };
template <class A, class B, class C>
__device__ __forceinline__ Stg3<A, B, C> restage(const Pub3<A, B, C>& v) {
    wave_sync();
    return Stg3<A, B, C>{{const_cast<A*>(v.a.p)}, {const_cast<B*>(v.b.p)}, {const_cast<C*>(v.c.p)}};
}

template <int L>
__device__ __forceinline__ uint64_t group_ballot(bool pred, int gbase) {
    uint64_t b = __ballot(pred);
    if constexpr (L == 64) {
        return b;
    } else {
        return (b >> gbase) & ((1ull << L) - 1ull);
    }
}

// Value of v held by lane `src` of this lane's group (src is group-uniform).
template <int L>
__device__ __forceinline__ float grp_get(float v, int src, int gbase) {
    if constexpr (L == 64) {
        return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
    } else {
        return __int_as_float(__builtin_amdgcn_ds_bpermute((gbase + src) << 2, __float_as_int(v)));
    }
}

template <int L>
__device__ __forceinline__ double grp_get(double v, int src, int gbase) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    if constexpr (L == 64) {
        return __hiloint2double(__builtin_amdgcn_readlane(hi, src),
                                __builtin_amdgcn_readlane(lo, src));
    } else {
        return __hiloint2double(__builtin_amdgcn_ds_bpermute((gbase + src) << 2, hi),
                                __builtin_amdgcn_ds_bpermute((gbase + src) << 2, lo));
    }
}

// ---- RNG ----------------------------------------------------------------------------------

// Box-Muller in double, rounded to float: (sine branch, cosine branch). log and sincos are the
// project's own (mh_math.h), bit-identical to the oracle's by construction.
__device__ __forceinline__ float2 box_muller_inl(unsigned int a, unsigned int b) {
    if (MH_ABLATE & 32) return make_float2((float)(a >> 8) * 0x1p-24f - 0.5f, (float)(b >> 8) * 0x1p-24f - 0.5f);
    const double u1 = (double)a * 0x1p-32 + 0x1p-33;
    const double u2 = (double)b * 0x1p-32 + 0x1p-33;
#if MH_ABLATE_OCML & 1
    const double rad = sqrt(-2.0 * ::log(u1));
#else
    const double rad = sqrt(-2.0 * mh_log(u1));
#endif
    const double ang = 6.283185307179586 * u2;
    double s, c;
#if MH_ABLATE_OCML & 1
    ::sincos(ang, &s, &c);
#else
    mh_sincos_medium(ang, &s, &c);  // (one argument reduction for both; ang < 2 pi)
#endif
    return make_float2((float)(rad * s), (float)(rad * c));
}

// Out of line so its log / sincos code is not duplicated at every call site.
static __device__ __attribute__((noinline)) float2 box_muller(unsigned int a, unsigned int b) {
    return box_muller_inl(a, b);
}

// rocRAND Philox4x32-10 stream of one chain. Words are taken a block of four at a time with
// rocrand4() (identical to four rocrand() calls from substate 0) and selected without dynamic
// register indexing, so the state stays in registers.
struct ChainRng {
    rocrand_state_philox4x32_10 st;
    uint4 buf;          // current block
    int idx;            // next word of buf (4 = exhausted)
    uint64_t draws;     // words consumed since draw 0
    int bm_has;
    float bm_val;

    __device__ __forceinline__ void init(uint64_t seed, uint64_t subsequence, uint64_t offset) {
        rocrand_init(seed, subsequence, offset & ~3ull, &st);
        buf = rocrand4(&st);
        idx = (int)(offset & 3);
        draws = offset;
    }
    __device__ __forceinline__ unsigned int next() {
        if (idx == 4) {
            buf = rocrand4(&st);
            idx = 0;
        }
        const unsigned int v = idx == 0 ? buf.x : idx == 1 ? buf.y : idx == 2 ? buf.z : buf.w;
        ++idx;
        ++draws;
        return v;
    }
    // curand_uniform stand-in (Kernel.cu:569,710): rocRAND's (0,1] float conversion.
    __device__ __forceinline__ float uniform() {
        return rocrand_device::detail::uniform_distribution(next());
    }
    // curand_normal stand-in (Kernel.cu:605,608,641): sine branch first, cosine branch cached
    // for the next call (cuRAND's caching order).
    __device__ __forceinline__ float normal() {
        if (bm_has) {
            bm_has = 0;
            return bm_val;
        }
        const unsigned int a = next();
        const unsigned int b = next();
        const float2 z = box_muller(a, b);
        bm_val = z.y;
        bm_has = 1;
        return z.x;
    }
};

// cuRAND's Box-Muller for curandStateXORWOW (curand_normal -> _curand_box_muller): float
// arithmetic on u = x * 2^-32 + 2^-33 and v = y * (2^-32 * 2pi_f) + half of that (one fma, as
// nvcc contracts it by default), s = sqrtf(-2 logf(u)), (sin(v) * s, cos(v) * s). logf, sinf
// and cosf are the double functions (mh_math.h) rounded once to float (the correctly rounded
// values but for ~2^-29 of inputs); NVIDIA's device path uses the approximate __sincosf, so its
// normals can differ in the last bits (DESIGN.md "RNG modes"). Out of line, like box_muller.
static __device__ __attribute__((noinline)) float2 curand_box_muller(unsigned int x, unsigned int y) {
    constexpr float kInv = 0x1p-32f;
    constexpr float kInv2Pi = 0x1p-32f * 6.2831855f;  // CURAND_2POW32_INV_2PI (exact scaling)
    const float u = (float)x * kInv + kInv * 0.5f;
    const float v = __builtin_fmaf((float)y, kInv2Pi, kInv2Pi * 0.5f);
    const float lg = (float)mh_log((double)u);
    const float s = __builtin_sqrtf(-2.0f * lg);
    double sn, cs;
    mh_sincos_medium((double)v, &sn, &cs);  // (v <= 2 pi)
    return make_float2((float)sn * s, (float)cs * s);
}

// cuRAND XORWOW stream (curandStateXORWOW_t; the reference seeds thread tid with
// curand_init(seed + tid, tid, 0), Kernel.cu:159,943): Marsaglia's xorshift over five words
// plus a Weyl sequence, 2^67 draws per subsequence. Seeding and the subsequence jump happen
// once per session in mh_xorwow_init_kernel; the state then lives in registers and is saved
// after every launch. Same interface as ChainRng.
struct ChainRngXw {
    unsigned int d, x0, x1, x2, x3, x4;
    uint64_t draws;
    int bm_has;
    float bm_val;

    __device__ __forceinline__ unsigned int next() {
        const unsigned int t = x0 ^ (x0 >> 2);
        x0 = x1;
        x1 = x2;
        x2 = x3;
        x3 = x4;
        x4 = (x4 ^ (x4 << 4)) ^ (t ^ (t << 1));
        d += 362437u;
        ++draws;
        return d + x4;
    }
    // curand_uniform (Kernel.cu:569,710): x * 2^-32 + 2^-33 in float, in (0, 1].
    __device__ __forceinline__ float uniform() { return (float)next() * 0x1p-32f + 0x1p-33f; }
    // curand_normal (Kernel.cu:605,608,641): sine branch first, cosine branch cached.
    __device__ __forceinline__ float normal() {
        if (bm_has) {
            bm_has = 0;
            return bm_val;
        }
        const unsigned int a = next();
        const unsigned int b = next();
        const float2 z = curand_box_muller(a, b);
        bm_val = z.y;
        bm_has = 1;
        return z.x;
    }
};

// The Philox stream of a chain that owns a whole wavefront (L = 64), drawn 64 words at a
// time: lane i holds word base + i and the Box-Muller pair of words (base + i, base + i + 1),
// so one pass of the double log / sincos serves every normal drawn from the window instead of
// one pass per normal. Draws read the window with v_readlane at the (uniform) draw index. The
// words and normals are exactly ChainRng's.
struct WaveWindow {
    unsigned int w;
    float bs, bc;
};

// Word d of a Philox stream: its block by rocrand4 (as ChainRng draws it) and the word picked
// without dynamic register indexing (that went through scratch).
__device__ __forceinline__ unsigned int philox_word(uint64_t seed, uint64_t subseq, uint64_t d) {
    rocrand_state_philox4x32_10 st;
    rocrand_init(seed, subseq, d & ~3ull, &st);
    const uint4 b = rocrand4(&st);
    const int q = (int)(d & 3);
    return q == 0 ? b.x : q == 1 ? b.y : q == 2 ? b.z : b.w;
}

// One window of WaveRng: lane i's word base + i and its Box-Muller pair.
__device__ __forceinline__ WaveWindow wave_window(uint64_t seed, uint64_t subseq, uint64_t at) {
    const int lane = __lane_id();
    WaveWindow ww;
    ww.w = philox_word(seed, subseq, at + (uint64_t)lane);
    const unsigned int w1 = (unsigned int)__shfl_down((int)ww.w, 1);  // lane 63's is unused
    const float2 z = box_muller_inl(ww.w, w1);
    ww.bs = z.x;
    ww.bc = z.y;
    return ww;
}

struct WaveRng {
    uint64_t seed, subseq;
    uint64_t base;   // first draw of the window
    uint64_t draws;  // next draw
    unsigned int w;  // lane i: word base + i
    float bs, bc;    // lane i: box_muller(word base + i, word base + i + 1)
    int bm_has;
    float bm_val;

    __device__ __forceinline__ void fill(uint64_t at) {
        base = at;
        const WaveWindow ww = wave_window(seed, subseq, at);
        w = ww.w;
        bs = ww.bs;
        bc = ww.bc;
    }
    // Called once per step (the only place a window is filled): starts a new window unless 16
    // draws remain in this one. A step that runs past the window (long frozen-object redraw
    // runs) draws the word directly instead.
    __device__ __forceinline__ void prepare() {
        if (draws - base > 64 - 16) fill(draws);
    }
    __device__ __forceinline__ unsigned int word_at(uint64_t d) const {
        if (d - base < 64) return (unsigned int)__builtin_amdgcn_readlane((int)w, (int)(d - base));
        return philox_word(seed, subseq, d);
    }
    __device__ __forceinline__ unsigned int next() { return word_at(draws++); }
    __device__ __forceinline__ float uniform() {
        return rocrand_device::detail::uniform_distribution(next());
    }
    __device__ __forceinline__ float normal() {
        if (bm_has) {
            bm_has = 0;
            return bm_val;
        }
        float zs, zc;
        if (draws - base < 63) {
            const int i = (int)(draws - base);
            zs = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bs), i));
            zc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bc), i));
        } else {
            // (inline: an out-of-line call here made the kernel spill across it)
            const float2 z = box_muller_inl(word_at(draws), word_at(draws + 1));
            zs = z.x;
            zc = z.y;
        }
        draws += 2;
        bm_val = zc;
        bm_has = 1;
        return zs;
    }
};

// WaveRng with the window's Box-Muller pairs in LDS (float[2][64] per chain, `bsl`) instead of
// two registers per lane: the full-evaluation step kernel is held to 96 VGPRs, and the pairs it
// kept in registers were spilled to scratch at every window fill.
struct WaveRngLds {
    // The stream's key and the window's first draw in LDS (ss[0] = seed, ss[1] = subsequence,
    // ss[2] = window start), read only at a window fill or a draw past the window; the step
    // carries only the 32-bit offset of the next draw in the window. The step kernel spills
    // scalar registers into vector lanes (v_writelane / v_readlane): the key out of scalar
    // registers took config 3 from 113.6 to 112.0 ms per launch, the offset for the 64-bit draw
    // count and window start from 111.7 to 110.3 ms (config 2 4.20 -> 4.01 ms with both).
    uint64_t* ss;
    __device__ __forceinline__ uint64_t seed_() const { return ss[0]; }
    __device__ __forceinline__ uint64_t subseq_() const { return ss[1]; }
    unsigned int off;  // next draw - window start
    unsigned int w;    // lane i: word (window start) + i
    float* bsl;        // [i], [64 + i]: box_muller(word start + i, word start + i + 1)
    int bm_has;
    float bm_val;

    __device__ __forceinline__ uint64_t draws() const { return ss[2] + off; }
    __device__ __forceinline__ void fill(uint64_t at) {
        // One lane stores the window start (64 lanes storing one address conflict in the LDS
        // banks; config 3 109.6 -> 109.3 ms per launch), and the wave_sync makes the other
        // lanes read it back: without it the compiler forwards each lane's stale value
        // (measured as forked chains).
        const int lane = __lane_id();
        if (lane == 0) ss[2] = at;
        wave_sync();
        off = 0;
        const WaveWindow ww = wave_window(seed_(), subseq_(), at);
        w = ww.w;
        bsl[lane] = ww.bs;
        bsl[64 + lane] = ww.bc;
    }
    __device__ __forceinline__ void prepare() {
        if (off > 64 - 16) fill(ss[2] + off);
    }
    __device__ __forceinline__ unsigned int word_off(unsigned int o) const {
        if (o < 64) return (unsigned int)__builtin_amdgcn_readlane((int)w, (int)o);
        return philox_word(seed_(), subseq_(), ss[2] + o);
    }
    __device__ __forceinline__ unsigned int next() { return word_off(off++); }
    __device__ __forceinline__ float uniform() {
        return rocrand_device::detail::uniform_distribution(next());
    }
    __device__ __forceinline__ float normal() {
        if (bm_has) {
            bm_has = 0;
            return bm_val;
        }
        float zs, zc;
        if (off < 63) {
            zs = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(bsl[off])));
            zc = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(bsl[64 + off])));
        } else {
            const float2 z = box_muller_inl(word_off(off), word_off(off + 1));
            zs = z.x;
            zc = z.y;
        }
        off += 2;
        bm_val = zc;
        bm_has = 1;
        return zs;
    }
};

template <class R> __device__ __forceinline__ uint64_t rng_draws(const R& r) { return r.draws; }
__device__ __forceinline__ uint64_t rng_draws(const WaveRngLds& r) { return r.draws(); }

template <bool XW, int L = 0> struct RngOf { using type = ChainRng; };
template <> struct RngOf<false, 64> { using type = WaveRng; };
template <int L> struct RngOf<true, L> { using type = ChainRngXw; };

template <class R> __device__ __forceinline__ void rng_prepare(R&) {}
__device__ __forceinline__ void rng_prepare(WaveRng& r) { r.prepare(); }

// Resume / save a chain's stream around a launch. Philox resumes from the draw count; XORWOW
// from its saved state words.
__device__ __forceinline__ void rng_load(ChainRng& r, const LaunchArgs& a, int64_t chain,
                                         const ChainMeta& m) {
    r.init(a.seed, (uint64_t)(a.chain_offset + chain), m.draws);
    r.bm_has = m.bm_has;
    r.bm_val = m.bm_val;
}
__device__ __forceinline__ void rng_load(ChainRngXw& r, const LaunchArgs& a, int64_t chain,
                                         const ChainMeta& m) {
    const unsigned int* w = a.xw + chain * 6;
    r.d = w[0];
    r.x0 = w[1];
    r.x1 = w[2];
    r.x2 = w[3];
    r.x3 = w[4];
    r.x4 = w[5];
    r.draws = m.draws;
    r.bm_has = m.bm_has;
    r.bm_val = m.bm_val;
}
__device__ __forceinline__ void rng_load(WaveRng& r, const LaunchArgs& a, int64_t chain,
                                         const ChainMeta& m) {
    r.seed = a.seed;
    r.subseq = (uint64_t)(a.chain_offset + chain);
    r.draws = m.draws;
    r.bm_has = m.bm_has;
    r.bm_val = m.bm_val;
    r.fill(m.draws);
}
__device__ __forceinline__ void rng_save(const WaveRng&, const LaunchArgs&, int64_t) {}
__device__ __forceinline__ void rng_prepare(WaveRngLds& r) { r.prepare(); }
// (bsl must be set before the load: the first window is filled here)
__device__ __forceinline__ void rng_load(WaveRngLds& r, const LaunchArgs& a, int64_t chain,
                                         const ChainMeta& m) {
    if (__lane_id() == 0) {
        r.ss[0] = a.seed;
        r.ss[1] = (uint64_t)(a.chain_offset + chain);
    }
    wave_sync();
    r.bm_has = m.bm_has;
    r.bm_val = m.bm_val;
    r.fill(m.draws);
}
__device__ __forceinline__ void rng_save(const WaveRngLds&, const LaunchArgs&, int64_t) {}
__device__ __forceinline__ void rng_save(const ChainRng&, const LaunchArgs&, int64_t) {}
__device__ __forceinline__ void rng_save(const ChainRngXw& r, const LaunchArgs& a, int64_t chain) {
    unsigned int* w = a.xw + chain * 6;
    w[0] = r.d;
    w[1] = r.x0;
    w[2] = r.x1;
    w[3] = r.x2;
    w[4] = r.x3;
    w[5] = r.x4;
}

// ---- numerics shared by every term ---------------------------------------------------------

// Kernel.cu:162-167: float difference, double root.
__device__ __forceinline__ double distance_f(float xi, float yi, float xj, float yj) {
    float fx = xi - xj;
    float fy = yi - yj;
    double dx = fx, dy = fy;
    double sq = dx * dx;
    sq = sq + dy * dy;
    return sqrt(sq);
}

// The shared transcendentals on the step kernels' rare paths (the exact terms of a step the
// rejection bound does not decide, Accept's threshold where the bound is open), as value-only
// helpers (arguments and result in registers). MH_MATH_OOL is a bit mask of the ones compiled
// out of line (1 atan2, 2 cosf, 4 exp), keeping their code and constants out of the step loop's
// register allocation; the others are inlined. Which wins is measured per kernel family.
#ifndef MH_MATH_OOL
#define MH_MATH_OOL 0  // (A/B, round 4: inlined is faster at configs 3 and 2; mh_delta.hip: 1)
#endif
#define MH_OOL_ATTR(bit) __attribute__((MH_OOL_KIND##bit))
#if MH_MATH_OOL & 1
#define MH_OOL_KIND1 noinline
#else
#define MH_OOL_KIND1 always_inline
#endif
#if MH_MATH_OOL & 2
#define MH_OOL_KIND2 noinline
#else
#define MH_OOL_KIND2 always_inline
#endif
#if MH_MATH_OOL & 4
#define MH_OOL_KIND4 noinline
#else
#define MH_OOL_KIND4 always_inline
#endif
#if MH_ABLATE_OCML & 2  // timing-only ablations: the device library's functions (results differ)
static __device__ MH_OOL_ATTR(1) double atan2_ool(double y, double x) { return ::atan2(y, x); }
#else
static __device__ MH_OOL_ATTR(1) double atan2_ool(double y, double x) { return mh_atan2(y, x); }
#endif
#if MH_ABLATE_OCML & 4
static __device__ MH_OOL_ATTR(2) float cos_f32_ool(float x) { return ::cosf(x); }
#else
static __device__ MH_OOL_ATTR(2) float cos_f32_ool(float x) { return mh_cos_f32(x); }
#endif
#if MH_ABLATE_OCML & 8
static __device__ MH_OOL_ATTR(4) double exp_ool(double x) { return ::exp(x); }
#else
static __device__ MH_OOL_ATTR(4) double exp_ool(double x) { return mh_exp(x); }
#endif

// Kernel.cu:170-182.
__device__ __forceinline__ double theta_f(float xi, float yi, float xj, float yj, float ti) {
    double dx = (double)(float)(xi - xj);
    double dy = (double)(float)(yi - yj);
    double tp = atan2_ool(dy, dx);
    if (tp < 0) tp = kTwoPI + tp;
    double t = tp - (double)ti;
    return (t < 0) ? kTwoPI + t : t;
}

// The reference's float atan2f / cosf, evaluated as the double function rounded once
// (mh_math.h, shared with the oracle).
__device__ __forceinline__ float atan2_f32(float y, float x) {
    return (float)atan2_ool((double)y, (double)x);
}
__device__ __forceinline__ float cos_f32(float x) { return cos_f32_ool(x); }

// minValue/maxValue (Kernel.cu:366-401) of a rectangle translated by (tx, ty), as floats.
__device__ __forceinline__ float4 shape_box(const RectShape& s, float tx, float ty) {
    float4 b;
    b.x = fminf(s.v0x, (float)(s.xmin1 + (double)tx));
    b.y = (float)(s.ymin + (double)ty);
    b.z = (float)(s.xmax + (double)tx);
    b.w = (float)(s.ymax + (double)ty);
    return b;
}

// calculateIntersectionArea, Kernel.cu:321-340 (boxes already rounded to float).
__device__ __forceinline__ float overlap(float4 a, float4 b) {
    float x5 = fmaxf(a.x, b.x);
    float y5 = fmaxf(a.y, b.y);
    float x6 = fminf(a.z, b.z);
    float y6 = fminf(a.w, b.w);
    if (x5 >= x6 || y5 >= y6) return 0.0f;
    return (x6 - x5) * (y6 - y5);
}

__device__ __forceinline__ float4 comp_overlaps(const DevRoom& rm, float4 box) {
    float4 t;
    t.x = overlap(box, make_float4(rm.comp[0][0], rm.comp[0][1], rm.comp[0][2], rm.comp[0][3]));
    t.y = overlap(box, make_float4(rm.comp[1][0], rm.comp[1][1], rm.comp[1][2], rm.comp[1][3]));
    t.z = overlap(box, make_float4(rm.comp[2][0], rm.comp[2][1], rm.comp[2][2], rm.comp[2][3]));
    t.w = overlap(box, make_float4(rm.comp[3][0], rm.comp[3][1], rm.comp[3][2], rm.comp[3][3]));
    return t;
}

__device__ __forceinline__ bool nonzero4(float4 t) {
    return t.x != 0.0f || t.y != 0.0f || t.z != 0.0f || t.w != 0.0f;
}

// Serially subtract, in lane order, the float4 terms of the group's lanes that are non-zero.
template <int L>
__device__ __forceinline__ float serial_sub4(float acc, float4 t, int gbase) {
    uint64_t bits = group_ballot<L>(nonzero4(t), gbase);
    while (bits) {
        int b = __builtin_ctzll(bits);
        bits &= bits - 1;
        acc = acc - grp_get<L>(t.x, b, gbase);
        acc = acc - grp_get<L>(t.y, b, gbase);
        acc = acc - grp_get<L>(t.z, b, gbase);
        acc = acc - grp_get<L>(t.w, b, gbase);
    }
    return acc;
}

template <int L>
__device__ __forceinline__ float serial_sub(float acc, float t, int gbase) {
    uint64_t bits = group_ballot<L>(t != 0.0f, gbase);
    while (bits) {
        int b = __builtin_ctzll(bits);
        bits &= bits - 1;
        acc = acc - grp_get<L>(t, b, gbase);
    }
    return acc;
}

template <int L>
__device__ __forceinline__ double serial_sub(double acc, double t, int gbase) {
    uint64_t bits = group_ballot<L>(t != 0.0, gbase);
    while (bits) {
        int b = __builtin_ctzll(bits);
        bits &= bits - 1;
        acc = acc - grp_get<L>(t, b, gbase);
    }
    return acc;
}

// One symmetry pair exactly as Kernel.cu:305-310 computes it, for the reflected row pose
// (rx, ry, rr) and object j's pose (xj, yj, ryj).
__device__ __forceinline__ float sym_val_exact(float xj, float yj, double ryj, float rx, float ry,
                                               double rr) {
    const float dp = (float)distance_f(xj, yj, rx, ry);
    float dt = (float)(ryj - rr);
    if (dt > kPI) dt = (float)((double)dt - kTwoPI);
    const float head = 5.0f - sqrtf(dp);
    return (float)((double)head - 0.4 * (double)fabsf(dt));
}

// fp32 estimate of sym_val_exact from q = {xf, yf, rotYf, -}: exact float differences,
// hardware (1 ulp) square roots, fp32 wrap and combine.
__device__ __forceinline__ float sym_val_fast(float4 q, float rx, float ry, float rr) {
    const float dx = q.x - rx;
    const float dy = q.y - ry;
    const float s = fmaf(dx, dx, dy * dy);
    const float h = __builtin_amdgcn_sqrtf(__builtin_amdgcn_sqrtf(s));
    float dt = q.z - rr;
    dt = (dt > 3.1416f) ? dt - 6.2832f : dt;
    return fmaf(-0.4f, fabsf(dt), 5.0f - h);
}

// Bound on |sym_val_fast - sym_val_exact| for an estimate v in a row with reflected angle rr,
// for poses with |x|, |y|, |rotY| < 1e15. Derivation (DESIGN.md "Symmetry estimate"): the
// square-root chain contributes <= 2^-21 (5 + |v|), the rotation difference and wrap <= 2^-22
// (12.6 + 2|v| + |rr|) x 0.4, the fp32 combine <= 2^-23 (15 + 2|v|) and the reference's own
// final rounding 2^-24 |v|; together < 2^-21 (12 + 2.2|v| + 0.1|rr|). A 4x margin gives:
__device__ __forceinline__ float sym_err(float v, float rr) {
#pragma clang fp contract(fast)  // (an allowance with a 4x margin: one rounding fewer is immaterial)
    return 0x1p-19f * (12.0f + 3.0f * fabsf(v) + fabsf(rr));
}

// ---- group collectives over the L lanes of one chain, in registers (DPP / permlane) ---------
//
// Butterfly partner at level OFF: lane ^ 1 and lane ^ 2 (DPP quad_perm), the mirrored quad /
// half-row for 4 and 8 (DPP row_half_mirror / row_mirror -- the same partner block as lane ^ OFF,
// which is all a reduction needs once values are uniform within each OFF-block), lane ^ 16 and
// lane ^ 32 (gfx950 v_permlane16_swap / v_permlane32_swap). None of them goes through LDS.
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF, bool BOUND_ZERO = false>
__device__ __forceinline__ int dpp_mov(int v, int old = 0) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROW_MASK, BANK_MASK, BOUND_ZERO);
}

template <int OFF>
__device__ __forceinline__ int bfly(int v) {
    if constexpr (OFF == 1) {
        return dpp_mov<0xB1>(v);   // quad_perm [1, 0, 3, 2]
    } else if constexpr (OFF == 2) {
        return dpp_mov<0x4E>(v);   // quad_perm [2, 3, 0, 1]
    } else if constexpr (OFF == 4) {
        return dpp_mov<0x141>(v);  // row_half_mirror
    } else if constexpr (OFF == 8) {
        return dpp_mov<0x140>(v);  // row_mirror
    } else if constexpr (OFF == 16) {
        const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return ((__lane_id() >> 4) & 1) ? (int)p[0] : (int)p[1];
    } else {
        const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (__lane_id() >> 5) ? (int)p[0] : (int)p[1];
    }
}

template <int OFF>
__device__ __forceinline__ float bfly(float v) {
    return __int_as_float(bfly<OFF>(__float_as_int(v)));
}

// Group-wide top two of (m1, m2) with the argmax of m1 (ties: lowest index, on every lane).
template <int L>
__device__ __forceinline__ void group_top2(float& m1, float& m2, int& j1) {
    auto level = [&](float p1, float p2, int pj) {
        const float lo = fminf(m1, p1);
        const bool take = p1 > m1 || (p1 == m1 && pj < j1);
        m2 = fmaxf(lo, fmaxf(m2, p2));
        m1 = fmaxf(m1, p1);
        j1 = take ? pj : j1;
    };
    level(bfly<1>(m1), bfly<1>(m2), bfly<1>(j1));
    level(bfly<2>(m1), bfly<2>(m2), bfly<2>(j1));
    if constexpr (L >= 8) level(bfly<4>(m1), bfly<4>(m2), bfly<4>(j1));
    if constexpr (L >= 16) level(bfly<8>(m1), bfly<8>(m2), bfly<8>(j1));
    if constexpr (L >= 32) level(bfly<16>(m1), bfly<16>(m2), bfly<16>(j1));
    if constexpr (L >= 64) level(bfly<32>(m1), bfly<32>(m2), bfly<32>(j1));
}

// Leader of a screened symmetry row from each lane's best two estimates (t1 at column tj, t2):
// the group maximum m, its column j, and whether it is clear -- held by one lane only, with
// every other estimate more than the two error bounds below m. Each lane tests its runner-up
// (t2 on the leader's lane, t1 elsewhere); its lower estimates are further away. One max
// butterfly and two ballots, where a top-two reduction moves three values per level.
struct SymLead {
    float m;
    int j;
    bool clear;
};

template <int L>
__device__ __forceinline__ SymLead group_sym_lead(float t1, float t2, int tj, int r, int gbase,
                                                  float rr) {
    float m = t1;
    if constexpr (L == 64) {
        // (one chain per wavefront: the row maxima by DPP, then row_bcast15 / row_bcast31 carry
        // them into lane 63, read as a scalar -- as wave_fsum, with -inf where a row is not
        // written; no permlane swaps)
        constexpr int NEG_INF = (int)0xff800000u;
        m = fmaxf(m, __int_as_float(dpp_mov<0xB1>(__float_as_int(m))));   // quad_perm [1,0,3,2]
        m = fmaxf(m, __int_as_float(dpp_mov<0x4E>(__float_as_int(m))));   // quad_perm [2,3,0,1]
        m = fmaxf(m, __int_as_float(dpp_mov<0x141>(__float_as_int(m))));  // row_half_mirror
        m = fmaxf(m, __int_as_float(dpp_mov<0x140>(__float_as_int(m))));  // row_mirror
        m = fmaxf(m, __int_as_float(dpp_mov<0x142, 0xA, 0xF, false>(__float_as_int(m), NEG_INF)));
        m = fmaxf(m, __int_as_float(dpp_mov<0x143, 0xC, 0xF, false>(__float_as_int(m), NEG_INF)));
        m = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m), 63));
    } else {
        m = fmaxf(m, bfly<1>(m));
        m = fmaxf(m, bfly<2>(m));
        if constexpr (L >= 8) m = fmaxf(m, bfly<4>(m));
        if constexpr (L >= 16) m = fmaxf(m, bfly<8>(m));
        if constexpr (L >= 32) m = fmaxf(m, bfly<16>(m));
    }
    // t1 is never NaN (it only takes values that compare greater), so some lane holds m.
    const uint64_t at = group_ballot<L>(t1 == m, gbase);
    const int lb = __builtin_ctzll(at);
    SymLead o;
    o.m = m;
    o.j = __float_as_int(grp_get<L>(__int_as_float(tj), lb, gbase));
    const float other = r == lb ? t2 : t1;
    const bool near = !(other == -INFINITY || m - other > sym_err(m, rr) + sym_err(other, rr));
    o.clear = o.j >= 0 && (at & (at - 1)) == 0 && group_ballot<L>(near, gbase) == 0;
    return o;
}

// Group-wide maximum of v with its index (ties: lowest index).
template <int L>
__device__ __forceinline__ void group_max_arg(float& v, int& j) {
    auto level = [&](float pv, int pj) {
        const bool take = pv > v || (pv == v && pj < j);
        v = take ? pv : v;
        j = take ? pj : j;
    };
    level(bfly<1>(v), bfly<1>(j));
    level(bfly<2>(v), bfly<2>(j));
    if constexpr (L >= 8) level(bfly<4>(v), bfly<4>(j));
    if constexpr (L >= 16) level(bfly<8>(v), bfly<8>(j));
    if constexpr (L >= 32) level(bfly<16>(v), bfly<16>(j));
    if constexpr (L >= 64) level(bfly<32>(v), bfly<32>(j));
}

// Group-wide integer max / sum.
template <int L>
__device__ __forceinline__ int group_max(int v) {
    v = max(v, bfly<1>(v));
    v = max(v, bfly<2>(v));
    if constexpr (L >= 8) v = max(v, bfly<4>(v));
    if constexpr (L >= 16) v = max(v, bfly<8>(v));
    if constexpr (L >= 32) v = max(v, bfly<16>(v));
    if constexpr (L >= 64) v = max(v, bfly<32>(v));
    return v;
}

template <int L>
__device__ __forceinline__ int group_sum(int v) {
    v += bfly<1>(v);
    v += bfly<2>(v);
    if constexpr (L >= 8) v += bfly<4>(v);
    if constexpr (L >= 16) v += bfly<8>(v);
    if constexpr (L >= 32) v += bfly<16>(v);
    if constexpr (L >= 64) v += bfly<32>(v);
    return v;
}

// Exclusive prefix sum over the group's lanes (r = lane within the group) and the group total.
// Inclusive scan by DPP row_shr within 16-lane rows (zero-filled at the row start, masked at an
// 8-lane group start), then row_bcast15 / row_bcast31 across rows.
template <int L>
__device__ __forceinline__ int group_excl_scan(int v, int r, int& total) {
    int x = v;
    int t = dpp_mov<0x111, 0xF, 0xF, true>(x);  // row_shr:1
    x += (r >= 1) ? t : 0;
    t = dpp_mov<0x112, 0xF, 0xF, true>(x);      // row_shr:2
    x += (r >= 2) ? t : 0;
    t = dpp_mov<0x114, 0xF, 0xF, true>(x);      // row_shr:4
    x += (r >= 4) ? t : 0;
    if constexpr (L >= 16) {
        t = dpp_mov<0x118, 0xF, 0xF, true>(x);  // row_shr:8
        x += t;
    }
    if constexpr (L >= 32) {
        t = dpp_mov<0x142, 0xA, 0xF, false>(x, 0);  // row_bcast15 into rows 1 and 3
        x += t;
    }
    if constexpr (L >= 64) {
        t = dpp_mov<0x143, 0xC, 0xF, false>(x, 0);  // row_bcast31 into rows 2 and 3
        x += t;
    }
    if constexpr (L == 64) {
        total = __builtin_amdgcn_readlane(x, 63);
    } else {
        total = __shfl(x, (__lane_id() & ~(L - 1)) + L - 1);
    }
    return x - v;
}

// a[m] for a runtime m, as a select chain (no dynamic register indexing).
template <int NPL, typename T>
__device__ __forceinline__ T sel(const T (&a)[NPL], int m) {
    T v = a[0];
#pragma unroll
    for (int q = 1; q < NPL; ++q) v = (m == q) ? a[q] : v;
    return v;
}

// ---- the rejection bound ---------------------------------------------------------------------
//
// Accept (Kernel.cu:706-713) rejects when u >= min(1, (float)exp(BETA (star - cur))). Most
// proposals are rejected, and a rejected proposal's costs are never used, so the exact,
// serially replayed sums are needed only when the decision is not already certain. The bound
// takes every term of every sum (each lane pre-sums the terms it holds), sums them across the
// chain's lanes in fp32 and bounds the distance to the reference's sequential sums: a sum of n
// non-zero terms accumulated with rounding unit U (one rounding, or a double rounding in float
// for the VisualBalance sums) is within n U sum|t| (1 + nU) of the exact sum; the fp32 group
// sum is within (k + 7) U sum|t| of it (k terms pre-summed per lane, a six-level tree, the
// conversion of double terms) -- all covered by (2n + 26 + k) U sum|t|. The cost composition
// (Kernel.cu:518-549) is bounded term by term with interval arithmetic (VisualBalance is
// 1-Lipschitz in its float coordinates, PairWise a product of two sums), every float rounding
// counted at 2U or more and the whole bound widened by 1.25. The decision is certain when the
// bound puts the upper total's exponent below log(u): u >= exp(x) (1 + U) >= (float)exp(x) for
// every total up to that bound.

// One lane's partial sums of the terms of Costs() for the bound, signed as the reference sums
// them; a* are partial sums of |term| where terms of both signs can occur.
struct BoundTerms {
    float nx, ny, anx, any;  // VisualBalance area * x, area * y (Kernel.cu:200-201)
    float fp, afp;           // FocalPoint -cos(phi) (:277)
    float sym;               // Symmetry -(row max) (:314), all <= 0
    float symw;              // sum of (n - i) |term i| over this lane's rows i (the sequential
                             // float sum's rounding weights, below); n |sym| is always valid
    float cl;                // Clearance -overlap (:429), all <= 0
    int kcl;                 // Clearance terms pre-summed by this lane
    float clpos;             // sum of pos |term| over this lane's Clearance terms at their
                             // positions pos in the non-zero list (0: no position credit)
    float sa;                // SurfaceArea -overlap (:463-479), all <= 0
    float pw, ang, aang;     // PairWise -(range term) (<= 0), PairWiseAngle (:222, :249-253)
    double pwd, angd;        // the same PairWise / PairWiseAngle partial sums in double
                             // (bound_decide<true>: the two sums in fp64)
    float efp;               // absolute error of this lane's FocalPoint terms (fp32 estimates)
    float eang;              // absolute error of this lane's PairWiseAngle terms (estimates)
    float esym;              // absolute error of this lane's Symmetry row maximum (an fp32
                             // estimate whose exact value the step has not needed yet)
    int pwx;                 // relative error of estimated PairWise terms, in U (uniform)
    int k;                   // most terms any lane pre-sums into any other partial sum (the
                             // same value on every lane: it enters the uniform bound)
};

// One butterfly level of a double: v + (its partner's v), both halves moved by bfly<OFF>.
template <int OFF>
__device__ __forceinline__ double bfly_add(double v) {
    return v + __hiloint2double(bfly<OFF>(__double2hiint(v)), bfly<OFF>(__double2loint(v)));
}

// One DPP level of a double: v + (the DPP source lane's v), both halves moved by dpp_mov (rows
// the row mask leaves out add 0).
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_add(double v) {
    return v + __hiloint2double(dpp_mov<CTRL, ROW_MASK, 0xF, false>(__double2hiint(v), 0),
                                dpp_mov<CTRL, ROW_MASK, 0xF, false>(__double2loint(v), 0));
}

// Sum of a double over the 64 lanes of the wavefront, uniform: the row sums by DPP (quad_perm,
// row_half_mirror, row_mirror), then row_bcast15 / row_bcast31 carry them into lane 63 -- six
// fp64 additions in a fixed order on the way to lane 63 (error <= 6 * 2^-53 * sum |v| beyond the
// lanes' own), as wave_fsum; no permlane swaps.
__device__ __forceinline__ double wave_dsum(double v) {
    v = dpp_add<0xB1>(v);   // quad_perm [1, 0, 3, 2]
    v = dpp_add<0x4E>(v);   // quad_perm [2, 3, 0, 1]
    v = dpp_add<0x141>(v);  // row_half_mirror
    v = dpp_add<0x140>(v);  // row_mirror
    v = dpp_add<0x142, 0xA>(v);  // row_bcast15 into rows 1 and 3
    v = dpp_add<0x143, 0xC>(v);  // row_bcast31 into rows 2 and 3
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63),
                            __builtin_amdgcn_readlane(__double2loint(v), 63));
}

// Sum of v over the 64 lanes of the wavefront, uniform (an SGPR): in-row butterflies (DPP
// quad_perm, row_half_mirror, row_mirror), then row_bcast15 / row_bcast31 carry the row sums
// into lane 63. The order is fixed, and the bound below counts six roundings per sum.
__device__ __forceinline__ float wave_fsum(float v) {
    v += __int_as_float(dpp_mov<0xB1>(__float_as_int(v)));   // quad_perm [1, 0, 3, 2]
    v += __int_as_float(dpp_mov<0x4E>(__float_as_int(v)));   // quad_perm [2, 3, 0, 1]
    v += __int_as_float(dpp_mov<0x141>(__float_as_int(v)));  // row_half_mirror
    v += __int_as_float(dpp_mov<0x140>(__float_as_int(v)));  // row_mirror
    v += __int_as_float(dpp_mov<0x142, 0xA, 0xF, false>(__float_as_int(v), 0));  // row_bcast15
    v += __int_as_float(dpp_mov<0x143, 0xC, 0xF, false>(__float_as_int(v), 0));  // row_bcast31
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Eight sums over the wavefront's 64 lanes at once, each returned uniform: a transposed
// butterfly whose levels halve the values a lane carries -- lane ^ 32 and lane ^ 16 by the gfx950
// permlane swaps (no selects: the swap pairs two values' halves), lane ^ 1 by DPP quad_perm --
// and then row rotations by 2, 4 and 8 add the eight lanes of a row that carry the same sum.
// Every sum is a six-level tree like wave_fsum's, in ~26 instructions for all eight instead of
// ~14 dependent ones each. Sum s ends on lane (s & 1) + 16 ((s >> 1) & 1) + 32 (s >> 2).
__device__ __forceinline__ void wave_fsum8(const float (&v)[8], float (&s)[8]) {
    float a[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // lanes 0-31: sum k; lanes 32-63: sum k + 4
        const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[k]),
                                                        __float_as_uint(v[k + 4]), false, false);
        a[k] = __uint_as_float(p[0]) + __uint_as_float(p[1]);
    }
    float b[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // rows 0..3: sums k, k + 2, k + 4, k + 6
        const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[k]),
                                                        __float_as_uint(a[k + 2]), false, false);
        b[k] = __uint_as_float(p[0]) + __uint_as_float(p[1]);
    }
    const bool odd = (__lane_id() & 1) != 0;  // even lanes keep b[0], odd lanes b[1]
    const float keep = odd ? b[1] : b[0], send = odd ? b[0] : b[1];
    float d = keep + __int_as_float(dpp_mov<0xB1>(__float_as_int(send)));  // quad_perm [1,0,3,2]
    d += __int_as_float(dpp_mov<0x122>(__float_as_int(d)));                // row_ror:2
    d += __int_as_float(dpp_mov<0x124>(__float_as_int(d)));                // row_ror:4
    d += __int_as_float(dpp_mov<0x128>(__float_as_int(d)));                // row_ror:8
    const int di = __float_as_int(d);
    s[0] = __int_as_float(__builtin_amdgcn_readlane(di, 0));
    s[1] = __int_as_float(__builtin_amdgcn_readlane(di, 1));
    s[2] = __int_as_float(__builtin_amdgcn_readlane(di, 16));
    s[3] = __int_as_float(__builtin_amdgcn_readlane(di, 17));
    s[4] = __int_as_float(__builtin_amdgcn_readlane(di, 32));
    s[5] = __int_as_float(__builtin_amdgcn_readlane(di, 33));
    s[6] = __int_as_float(__builtin_amdgcn_readlane(di, 48));
    s[7] = __int_as_float(__builtin_amdgcn_readlane(di, 49));
}

// A wave-uniform float, in a scalar register.
__device__ __forceinline__ float uniform_f(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// An interval of fp32 totals (a chain's current total is an exact value, lo == hi, or, after a
// proposal accepted on the bound alone, the bound's interval around the exact total).
struct CostIv {
    float lo, hi;
};

enum { BOUND_OPEN = 0, BOUND_REJECT = 1, BOUND_ACCEPT = 2 };

// Whether Accept's decision for this proposal is already certain, for a chain that owns the
// wavefront: BOUND_REJECT / BOUND_ACCEPT, or BOUND_OPEN (the exact costs are needed). n objects,
// c clearances, nrel relationships, ncl non-zero Clearance terms; `cur` holds the current
// total. The arithmetic after the lane sums is fp32 on wave-uniform values (with DPW the
// PairWise and PairWiseAngle sums and their product are fp64: their fp32 error dominated the
// bound at N = 256, where PairWise is most of the total); the proposal's exact total lies in
// t +- 1.25 e. `star` receives an interval around it that also absorbs the rounding of its own
// ends (e >= 8 U |t|, so 0.25 e does).
//
// e is the sum of term-by-term error bounds: each sum's (the reference's sequential rounding
// and this estimate's), each composition step of Costs() (the e1, e2 and 12 U terms), and the
// roundings no term covers -- the reference's five float additions of the total (:547), each
// at most U times a partial sum of the components, whose magnitudes add up to at most cabs
// below; the two additions forming t; the weight products' second rounding (e1 and e2 count
// three of the four roundings of W * component on either side); and the decision's own
// arithmetic on t, e and cur (t + 1.25 e, minus cur, the star ends): 8 U cabs + 3 U (|o1| +
// |o2|) + 3 U (|t| + |cur|) covers them.
// The lane parts of the eight sums bound_decide composes, from this lane's terms (below). Each
// part is a sum of per-component contributions, so lanes (or wavefronts) holding different
// components of one configuration may each call it with the others' fields zero and add their
// parts (the speculative kernel's two wavefronts per node): the additions' extra roundings stay
// within the tree allowance's six levels. `part[7]` takes the angle allowances scaled by 1 / cr.
template <bool DPW = false>
__device__ __forceinline__ void bound_parts(const DevRoom& rm, int n, int c, int nrel, int ncl,
                                            const BoundTerms& bt, float (&part)[8]) {
#pragma clang fp contract(fast)
    constexpr float U = 0x1p-24f;
    const float kf = (float)bt.k;
    const float lfp = rm.w_fp * bt.fp, lsym = rm.w_sym * bt.sym, lcl = rm.w_cl * bt.cl,
                lsa = rm.w_sa * bt.sa;
    const float lin = (lfp + lsym) + (lcl + lsa);
    const float afp = fabsf(rm.w_fp) * bt.afp;
    const float alin = afp + fabsf(lsym) + fabsf(lcl) + fabsf(lsa);  // (lanes' |components|)
    // A sequential sum of m terms in a float accumulator (Symmetry :314, Clearance :429) is
    // within U sum_q |partial sum q| (1 + m U) of the exact sum: one rounding to nearest per
    // add, and zero terms do not round. With terms of one sign the partial sums add up to
    // sum_q (m - q) |t_q|, t_q the term at position q: per lane, symw, and ncl |cl| - clpos for
    // the compacted Clearance terms (clpos = 0 gives the plain m U sum |t|). In a double
    // accumulator (FocalPoint, PairWise, PairWiseAngle) the same is m 2^-53 sum |t| (eacc, in
    // units of U). This estimate: terms rounded to float once, k pre-summed per lane, a
    // six-level tree: (k + 7) U sum |t|. "26" covers the second-order parts for m < 2^20.
    const float eacc = 0x1p-29f * (float)(n + nrel);
    const float wsym = fabsf(rm.w_sym) * bt.symw;
    const float wcl = fabsf(rm.w_cl) * fmaxf(0.0f, (float)ncl * fabsf(bt.cl) - bt.clpos);
    const float elin = (26.0f + kf + eacc) * U * afp + (26.0f + kf) * U * fabsf(lsym) +
                       U * wsym + (26.0f + (float)bt.kcl) * U * fabsf(lcl) + U * wcl +
                       (4.0f * (c + n) + 26.0f + kf) * U * fabsf(lsa) + 12.0f * U * alin +
                       fabsf(rm.w_fp) * bt.efp + fabsf(rm.w_sym) * bt.esym;
    // (fp32 path: the PairWise sum's relative allowance, estimates included; the angle terms'
    // absolute allowances enter its magnitude sum scaled by 1 / cr, so eang = cr a_ang covers them)
    const float cr32 = (26.0f + kf + eacc + (float)bt.pwx) * U;
    // sum[6] bounds sum |area x| and sum |area y| for VisualBalance; the components' sum of
    // magnitudes (alin, for the catch-all term) rides along in sum[7] with the angle terms'
    // magnitudes when their sum is fp64 (DPW: sum[7] then only scales a 2^-53 error), in sum[6]
    // otherwise
    // (eang / cr32 from the hardware reciprocal, 1 ulp, raised by 8 U: never below the quotient)
    const float icr = __builtin_amdgcn_rcpf(cr32) * (1.0f + 8.0f * U);
    part[0] = bt.nx;
    part[1] = bt.ny;
    part[2] = bt.pw;
    part[3] = bt.ang;
    part[4] = lin;
    part[5] = elin;
    part[6] = bt.anx + bt.any + (DPW ? 0.0f : alin);
    part[7] = bt.aang + (DPW ? alin : bt.eang * icr);
}

// The proposal's total estimate and decision from the eight sums of bound_parts (fp32 path:
// the PairWise and PairWiseAngle sums in sum[2], sum[3]; with DPW their fp64 sums come from the
// wavefront's lanes' bt.pwd, bt.angd, and the estimated angle terms' allowances from bt.eang).
// Returns BOUND_REJECT / BOUND_ACCEPT / BOUND_OPEN for this lane (the caller makes it uniform)
// and the proposal's interval in `star`.
template <bool DPW = false>
__device__ __forceinline__ float bound_te(const DevRoom& rm, int n, int nrel, int k, int pwx,
                                          const float (&sum)[8], const BoundTerms& bt, CostIv cur,
                                          float slack, float& e_out) {
#pragma clang fp contract(fast)
    constexpr float U = 0x1p-24f;
    const float kf = (float)k;
    const float eacc = 0x1p-29f * (float)(n + nrel);
    const float cr32 = (26.0f + kf + eacc + (float)pwx) * U;
    const float s_nx = sum[0], s_ny = sum[1], s_lin = sum[4], s_elin = sum[5];
    const float a_nx = fmaxf(fabsf(s_nx), sum[6]), a_ny = fmaxf(fabsf(s_ny), sum[6]),
                a_ang = fmaxf(fabsf(sum[3]), sum[7]);
    // VisualBalanceCosts (Kernel.cu:191-207): -|(nx/denom, ny/denom) - centroid/2|
    const float id = fabsf(rm.inv_denom);
    const float cv = (n + 26.0f + kf) * U;  // (float accumulators, Kernel.cu:200-201)
    // The chain of the reference's roundings below -- (enx + eny) = S for the two sums, 3 U on
    // ad, bd (the division), 2 U on fx, fy (the centroid subtraction), 3 U on the distance (the
    // reference's correctly rounded root, U, and this estimate's 1-ulp hardware root, 2 U), 3 U
    // on the weight product -- composed with each (1 + kU) factor expanded: the exact error of
    // w_vb vb is at most |w_vb| (S (1 + 12 U) + 3.01 U A + 2.01 U F + 7 U |vb|), A = |ad| + |bd|,
    // F = |fx| + |fy|; written with 32 U, 4 U, 4 U and 8 U to absorb this expression's own roundings.
    const float S = cv * id * (a_nx + a_ny);
    const float ad = s_nx * rm.inv_denom, bd = s_ny * rm.inv_denom;
    const float fx = ad - rm.cxf, fy = bd - rm.cyf;
    const float vb = -__builtin_amdgcn_sqrtf(fx * fx + fy * fy);
    const float o2 = rm.w_vb * vb;
    // (+ 2^-40: a root of a denormal argument, where the hardware root's 1 ulp is not promised,
    // is below 2^-60)
    const float e2 = fabsf(rm.w_vb) *
                     (S * (1.0f + 32.0f * U) +
                      4.0f * U * ((fabsf(ad) + fabsf(bd)) + (fabsf(fx) + fabsf(fy)) + 2.0f * fabsf(vb)) +
                      0x1p-40f);
    // PairWise x PairWiseAngle (Kernel.cu:518), both sums accumulated in double (:222, :249-253)
    float pa, dpa;
    if constexpr (DPW) {
        // fp64 lane partial sums and tree: within (k + 8) 2^-53 sum |t| of the exact sums, the
        // reference's within nrel 2^-53 sum |t|; the product rounded once to double and then,
        // like the reference's (float)(pw * ang), to float
        const double spw = wave_dsum(bt.pwd), sang = wave_dsum(bt.angd);
        const double pad = spw * sang;
        const float cr = (float)((double)(nrel + k + 12) * 0x1p-53);
        float epw = cr * (float)fabs(spw) * (1.0f + 64.0f * U),
              eang = cr * a_ang * (1.0f + 64.0f * U);
        if (pwx) {  // (uniform) estimated relationship terms (the incremental kernel's
                    // EstState): kPwEstU U relative on PairWise, eang each on the angles; the
                    // fp32 tree sum of the allowances raised by 8 U, 64 U on the relative part
            epw += (float)pwx * U * (float)fabs(spw) * (1.0f + 64.0f * U);
            eang += wave_fsum(bt.eang) * (1.0f + 8.0f * U);
        }
        pa = (float)pad;
        dpa = (float)fabs(spw) * eang + (float)fabs(sang) * epw + epw * eang +
              (float)(0x1p-52 * fabs(pad));
    } else {
        const float s_pw = sum[2], s_ang = sum[3];
        const float epw = cr32 * fabsf(s_pw), eang = cr32 * a_ang;  // (double accumulators)
        pa = s_pw * s_ang;
        dpa = fabsf(s_pw) * eang + fabsf(s_ang) * epw + epw * eang;
    }
    const float o1 = rm.w_pw * pa;
    const float e1 = fabsf(rm.w_pw) * (dpa + 3.0f * U * (fabsf(pa) + dpa));
    // total (Kernel.cu:547) and its ends
    const float t = (o1 + o2) + s_lin;
    const float acur = fmaxf(fabsf(cur.lo), fabsf(cur.hi));
    const float cabs = fabsf(o1) + e1 + fabsf(o2) + e2 + (DPW ? sum[7] : sum[6]);
    e_out = slack * (e1 + e2 + s_elin + 3.0f * U * (fabsf(o1) + fabsf(o2)) +
                     8.0f * U * cabs + 3.0f * U * (fabsf(t) + acur));
    return t;
}

// Accept's decision for a proposal whose exact total lies in t +- 1.25 e (bound_te, e computed
// for a current total of the magnitude of `cur`'s: the decision's own arithmetic on it), against
// the current total's interval `cur`; the proposal's interval in `star` (below).
__device__ __forceinline__ int bound_vs(float t, float e, float u, CostIv cur, CostIv& star) {
#pragma clang fp contract(fast)
    const float x = (float)kBeta * ((t + 1.25f * e) - cur.lo);   // beta (star - cur), upper end
    const float xl = (float)kBeta * ((t - 1.25f * e) - cur.hi);  // and lower end
    // log(u) from the f32 log: within 1e-5 of the true value for u in [2^-33, 1]; 1e-4 margin
    const float lu = __logf(u);
    // Reject: x <= lu - 1e-4 (the compares are NaN-false: an invalid bound is never certain).
    // Accept: the threshold min(1, exp(beta (star - cur))) is at most 1, so u == 1.0f (which
    // the (0, 1] uniform draws, ~2^-25 of draws) is never accepted; otherwise the threshold is 1
    // for beta (star - cur) >= 0, and exp(beta (star - cur)) (> exp(-24)) exceeds u when
    // log(u) < xl - 1e-4. (Round 2 accepted u == 1.0f whenever xl > 1e-4: a certain ACCEPT
    // against Accept's rejection, found by tools/bound_check.py.)
    const bool rej = x <= lu - 1e-4f && x > -1e30f;
    const bool acc = u < 1.0f && (xl >= 0.0f || (xl > -23.9f && lu < xl - 1e-4f));
    star.lo = t - 1.5f * e;
    star.hi = t + 1.5f * e;
    return rej ? BOUND_REJECT : (acc ? BOUND_ACCEPT : BOUND_OPEN);
}

template <bool DPW = false>
__device__ __forceinline__ int bound_compose(const DevRoom& rm, int n, int nrel, int k, int pwx,
                                             const float (&sum)[8], const BoundTerms& bt, float u,
                                             CostIv cur, CostIv& star, float slack) {
    float e;
    const float t = bound_te<DPW>(rm, n, nrel, k, pwx, sum, bt, cur, slack, e);
    return bound_vs(t, e, u, cur, star);
}

// Whether Accept's decision for this proposal is already certain, for a chain that owns the
// wavefront: BOUND_REJECT / BOUND_ACCEPT, or BOUND_OPEN (the exact costs are needed). n objects,
// c clearances, nrel relationships, ncl non-zero Clearance terms; `cur` holds the current
// total. The arithmetic after the lane sums is fp32 on wave-uniform values (with DPW the
// PairWise and PairWiseAngle sums and their product are fp64: their fp32 error dominated the
// bound at N = 256, where PairWise is most of the total); the proposal's exact total lies in
// t +- 1.25 e. `star` receives an interval around it that also absorbs the rounding of its own
// ends (e >= 8 U |t|, so 0.25 e does).
//
// e is the sum of term-by-term error bounds: each sum's (the reference's sequential rounding
// and this estimate's), each composition step of Costs() (the e1, e2 and 12 U terms), and the
// roundings no term covers -- the reference's five float additions of the total (:547), each
// at most U times a partial sum of the components, whose magnitudes add up to at most cabs
// below; the two additions forming t; the weight products' second rounding (e1 and e2 count
// three of the four roundings of W * component on either side); and the decision's own
// arithmetic on t, e and cur (t + 1.25 e, minus cur, the star ends): 8 U cabs + 3 U (|o1| +
// |o2|) + 3 U (|t| + |cur|) covers them. (The arithmetic: bound_parts and bound_compose.)
template <bool DPW = false>
__device__ __forceinline__ int bound_decide(const DevRoom& rm, int n, int c, int nrel, int ncl,
                                            const BoundTerms& bt, float u, CostIv cur,
                                            CostIv& star, float slack = 1.0f) {
    float part[8], sum[8];
    bound_parts<DPW>(rm, n, c, nrel, ncl, bt, part);
    wave_fsum8(part, sum);
    const int d = bound_compose<DPW>(rm, n, nrel, bt.k, bt.pwx, sum, bt, u, cur, star, slack);
    // the chain's first lane decides, so the decision is wave-uniform by construction
    return __builtin_amdgcn_readfirstlane(d);
}

// Whether Accept certainly rejects this proposal (bound_decide with an exact current total).
__device__ __forceinline__ bool certain_reject(const DevRoom& rm, int n, int c, int nrel, int ncl,
                                               const BoundTerms& bt, float u, float cur,
                                               float slack = 1.0f) {
    CostIv star;
    return bound_decide(rm, n, c, nrel, ncl, bt, u, CostIv{cur, cur}, star, slack) ==
           BOUND_REJECT;
}

// Exact row maxima of the symmetry rows this lane owns (rows m * L + r), with the column that
// attains each (-1: the 0 floor of Kernel.cu:303 is the maximum).
template <int NPL>
struct SymRows {
    float mx[NPL];
    int arg[NPL];
};

// Non-zero Clearance pairs of a configuration, for the incremental pair update of the
// full-evaluation step (one object per lane): this lane's column mask (bit i: clearance i
// overlaps the lane's object) and which of the two LDS row-word buffers holds the rows.
struct ClPairs {
    uint64_t cm;
    int buf;
    double rpw, rang;  // this lane's relationship terms (kept for relationships a move misses)
    float cph;         // this lane's object's cos(phi) (kept for objects a move misses)
    float4 sac;        // SurfaceArea overlaps of clearance `lane` at object `lane`'s pose
    bool dc, dr;       // cph / rpw, rang hold fp32 estimates, not the reference's values (steps
                       // the rejection bound decides compute only those; an exact pass fixes
                       // them when a step needs the exact sums)
    float eang;        // the allowance of an estimated rang
    float clc;         // the rejection bound's Clearance partial sum of this lane's object
                       // (its column, clearances in order): recomputed only when it may change
};

// Allowances of the fp32 estimates of the FocalPoint and relationship terms (mh_chain.hip
// approx_terms): |cos(phi) estimate - the reference's float| <= kDeltaCph, theta's estimate
// within kDeltaTh of the reference's double, the PairWise term within kPwEstU U relative. The
// check build verifies every estimate against the exact value (sites 30-32).
//   theta: atan2_est within 2^-20 (below), the wrap's + 2pi and the rotation's subtraction each
//   rounded at |values| < 32 (the callers require |rotY| < 16): 3 x 2^-20 more, so 2^-18 in all.
//   cos(phi): the angle as above plus the reference's own float roundings of at, b and phi
//   (|phi| < 16: 2^-20 each), cos_est within 2^-22: under 2^-17.4.
//   PairWise: the distance within 3 U (float squares and sum, a 1-ulp square root), 1 / start
//   and (float) end within U each, the products U each, the hardware reciprocal 2 U: f within
//   7 U, f * f within 15 U + O(U^2).
// (kDeltaCph, kDeltaTh, kPwEstU: mh_device.h, shared with the host's estimate constants)

// atan2(y, x) in fp32 for the rejection bound's estimates: the octant reduction t = min / max
// (hardware reciprocal, 1 ulp), an odd degree-15 polynomial fitted to atan on [0, 1] (2^-23 in
// fp32 Horner form), then pi/2 - a, pi - a and y's sign. Within 2^-21.3 of atan2 over 4e7
// random and near-diagonal pairs (numpy emulation with the reciprocal 1 ulp off either way), so
// 2^-20 is the figure the allowances use. Requires max(|x|, |y|) >= 2^-100 (callers check: a
// zero vector or a denormal maximum would meet the reciprocal's flush).
__device__ __forceinline__ float atan2_est(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float t = mn * __builtin_amdgcn_rcpf(mx);
    const float s = t * t;
    float p = -0.0040545351803302765f;
    p = __builtin_fmaf(p, s, 0.021862849593162537f);
    p = __builtin_fmaf(p, s, -0.05591217800974846f);
    p = __builtin_fmaf(p, s, 0.09642186760902405f);
    p = __builtin_fmaf(p, s, -0.1390862613916397f);
    p = __builtin_fmaf(p, s, 0.19946564733982086f);
    p = __builtin_fmaf(p, s, -0.33329859375953674f);
    p = __builtin_fmaf(p, s, 0.9999993443489075f);
    float a = p * t;
    a = ay > ax ? 1.5707963705062866f - a : a;
    a = x < 0.0f ? 3.1415927410125732f - a : a;
    return __builtin_copysignf(a, y);
}

// cos(x) in fp32 for |x| < 16 (callers check): x - k pi/2 by a two-constant fused reduction
// (within 2^-24), sin / cos polynomials fitted on [-pi/4, pi/4] (2^-24 in fp32), the quadrant's
// sign and choice. Within 2^-22 of cos(x).
__device__ __forceinline__ float cos_est(float x) {
    const float k = __builtin_rintf(x * 0.63661977236758134f);
    float r = __builtin_fmaf(-k, 1.5707963705062866f, x);
    r = __builtin_fmaf(-k, -4.37113882867379e-08f, r);
    const float s = r * r;
    const float ps = __builtin_fmaf(__builtin_fmaf(s, -0.00019488755788188428f,
                                                   0.008331923745572567f), s, -0.16666649281978607f);
    const float sn = __builtin_fmaf(r * s, ps, r);
    const float pc = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(s, 2.438225783407688e-05f,
                                                                  -0.0013886678498238325f),
                                                   s, 0.04166661947965622f),
                                    s, -0.5f);
    const float cs = __builtin_fmaf(s, pc, 1.0f);
    const int q = (int)k;
    const float v = (q & 1) ? sn : cs;
    return ((q + 1) & 2) ? -v : v;
}

// (rel_est_consts: mh_device.h, shared with the host)

// The fp32 PairWise estimate of a relationship from its objects' pose words (the reference's float
// differences; the distance within 3 U of the reference's double), setting `amb` near the range's
// ends. e0 = {(float)start, (float)end, 1 / start, -} (rel_est_consts); within kPwEstU U relative.
__device__ __forceinline__ double rel_pw_est(float4 e0, ObjP ps, ObjP pt, bool& amb) {
#pragma clang fp contract(fast)  // (fused: fewer roundings than the allowance counts)
    constexpr float U = 0x1p-24f;
    const float fx = ps.xf - pt.xf, fy = ps.yf - pt.yf;
    const float d2 = fx * fx + fy * fy;
    const float d = __builtin_amdgcn_sqrtf(d2);  // (1 ulp)
    const float st = e0.x, en = e0.y;
    amb |= !(d2 >= 0x1p-100f) || fabsf(d - st) <= 8.0f * U * fabsf(st) ||
           fabsf(d - en) <= 8.0f * U * fabsf(en);
    const float f = d < st ? d * e0.z : (d > en ? en * __builtin_amdgcn_rcpf(d) : 0.0f);
    return (double)(f * f);
}

// The fp32 PairWiseAngle estimate from theta's estimate `tp` (atan2_est) and the target's pose
// words, with its absolute allowance `eang`; `amb` near theta's wraps and the wrapped range's
// switch, for a target rotation outside |rotY| < 16, or where the relationship takes no estimate.
// e1 = {(float)amin, (float)amax, 1 / norm, flags}, ea = e0.w (rel_est_consts). `flat`: the pair's
// float y difference is zero and its x difference positive, so theta is exactly +-0 (atan2 of a
// zero over a positive number, Kernel.cu:171-176) and takes no wrap: tp = 0 is then no ambiguity.
__device__ __forceinline__ double rel_ang_est(float4 e1, float ea, ObjP atp, float tp, float& eang,
                                              bool& amb, bool flat = false) {
#pragma clang fp contract(fast)  // (fused: fewer roundings than the allowance counts)
    constexpr float U = 0x1p-24f, Y = (float)kTwoPI;
    const int fl = __float_as_int(e1.w);
    amb |= (fl & RE_EXACT) != 0 || !(fabsf(atp.rotYf) < 16.0f) || (!flat && fabsf(tp) <= kDeltaTh);
    if (tp < 0.0f) tp = tp + Y;
    const float t = tp - atp.rotYf;
    amb |= fabsf(t) <= kDeltaTh;
    const float th = t < 0.0f ? t + Y : t;
    bool on;
    if (fl & RE_WRAP) {
        // fmodf(x, 2pi) for x in [0, 4pi) is x or x - 2pi, exact (Sterbenz); outside: exact terms
        const float x = e1.x + th;
        amb |= !(x >= 0.0f && x < 2.0f * Y);
        const float w = x >= Y ? x - Y : x;
        amb |= fabsf(w - e1.y) <= 2.0f * kDeltaTh || fabsf(w) <= 2.0f * kDeltaTh ||
               fabsf(w - Y) <= 2.0f * kDeltaTh;
        on = w > e1.y;
    } else {
        on = e1.x < th || th < e1.y;  // (continuous at its switch)
    }
    const float v = on ? fminf(fabsf(th - e1.x), fabsf(th - e1.y)) * e1.z : 0.0f;
    eang = ea + 4.0f * U * fabsf(v);
    return (double)v;
}

// the focal term's estimate from the focal angle's estimate `at` (Kernel.cu:271, 277)
__device__ __forceinline__ float cph_est(float at, ObjP p, bool& ambo) {
    const float ph = (at - p.rotYf) + (float)kHalfPI;
    ambo |= !(fabsf(p.rotYf) < 16.0f) || !(fabsf(ph) < 16.0f);
    return cos_est(ph);
}


// PairWiseCosts (:210-233) and PairWiseAngleCosts (:236-263) terms of relationship q.
// Split form for callers that batch the atan2: rel_pair() gives the PairWise term and theta's
// atan2 arguments (and the target's rotation), rel_angle() the angle term from that atan2.
__device__ __forceinline__ double rel_pair(const RelConst& rc, const ObjP* P, double& dy,
                                           double& dx, float& ti) {
    double tpw = 0.0;
    const ObjP ps = P[rc.s], pt = P[rc.t];
    const double d = distance_f(ps.xf, ps.yf, pt.xf, pt.yf);
    // d / start below the range, end / d above it: one division for either side
    const bool below = d < rc.start, above = d > rc.end;
    if (below || above) {
        const double f = (below ? d : rc.end) / (below ? rc.start : d);
        tpw = f * f;
    }
    const ObjP as = P[rc.as], at = P[rc.at];
    dx = (double)(float)(as.xf - at.xf);  // theta(), Kernel.cu:170-182
    dy = (double)(float)(as.yf - at.yf);
    ti = at.rotYf;
    return tpw;
}

__device__ __forceinline__ double rel_angle(const RelConst& rc, double tp, float ti) {
    if (tp < 0) tp = kTwoPI + tp;
    const double t = tp - (double)ti;
    const double th = (t < 0) ? kTwoPI + t : t;
    bool on;
    double norm;
    if (rc.amin > rc.amax) {
        float w = fmodf((float)(rc.amin + th), (float)kTwoPI);
        on = (double)w > rc.amax;
        norm = rc.norm_w;
    } else {
        on = rc.amin < th || th < rc.amax;
        norm = rc.norm_n;
    }
    return on ? fmin(fabs(th - rc.amin), fabs(th - rc.amax)) / norm : 0.0;
}

// `pose(k)` gives object k's float pose words (ObjP: xf, yf, rotYf).
template <class PoseOf>
__device__ __forceinline__ void rel_terms_of(const RelConst& rc, PoseOf pose, double& tpw,
                                             double& tang) {
    tpw = 0.0;
    tang = 0.0;
    const ObjP ps = pose(rc.s), pt = pose(rc.t);
    const double d = distance_f(ps.xf, ps.yf, pt.xf, pt.yf);
    // d / start below the range, end / d above it: one division for either side
    const bool below = d < rc.start, above = d > rc.end;
    if (below || above) {
        const double f = (below ? d : rc.end) / (below ? rc.start : d);
        tpw = f * f;
    }
    const ObjP as = pose(rc.as), at = pose(rc.at);
    const double th = theta_f(as.xf, as.yf, at.xf, at.yf, at.rotYf);
    bool on;
    double norm;
    if (rc.amin > rc.amax) {
        float w = fmodf((float)(rc.amin + th), (float)kTwoPI);
        on = (double)w > rc.amax;
        norm = rc.norm_w;
    } else {
        on = rc.amin < th || th < rc.amax;
        norm = rc.norm_n;
    }
    if (on) tang = fmin(fabs(th - rc.amin), fabs(th - rc.amax)) / norm;
}

__device__ __forceinline__ void rel_terms(const RelConst& rc, const ObjP* P, double& tpw,
                                          double& tang) {
    rel_terms_of(rc, [P](int k) { return P[k]; }, tpw, tang);
}

// ---- proposal draws and the accept rule ----------------------------------------------------

template <class Rng>
__device__ __forceinline__ int rand_int(Rng& rng, int max, int min) {
    float u = rng.uniform();
    u = (float)((double)u * ((double)(max - min) + 0.999999));
    u = u + (float)min;
    return (int)truncf(u);
}

template <class Rng>
__device__ __forceinline__ int pick_object(Rng& rng, int n, const unsigned char* frozen) {
    int k = rand_int(rng, n - 1, 0);
    while (frozen[k]) k = rand_int(rng, n - 1, 0);  // frozen[n] == 1: index n is redrawn
    return k;
}


// Accept(), Kernel.cu:706-713 (maximisation, BETA = 2).
// The threshold min(1, (float)exp(x)) of Accept without evaluating exp where it is decided:
// x >= 0 gives exp(x) >= 1, so the threshold is exactly 1; x < -24 gives (float)exp(x) <
// 3.8e-11, below every uniform either stream draws (>= 2^-33), so any u rejects -- 0 decides
// the same. (The uniform is drawn in every case, so the stream is unchanged.)
__device__ __forceinline__ float accept_threshold(double x) {
    if (x >= 0.0) return 1.0f;
    if (x < -24.0) return 0.0f;
    return fminf(1.0f, (float)exp_ool(x));
}

// Accept's decision u < accept_threshold(x), screened in fp32. For -24 <= x < 0, e = v_exp_f32(
// (float)x log2(e)) is within 4e-6 relative of exp(x): (float)x is off by at most 2^-20, the
// product's rounding by 2^-24 * 35, log2(e)'s by 2^-25 relative, v_exp_f32 by 1 ulp. A u more
// than 1e-4 relative below e is then below exp(x) (1 - 2^-24) <= (float)exp(x), and one more
// than 1e-4 above is above (float)exp(x): decided without the double exp; only a u inside that
// band (about 2e-4 of the draws near a threshold) evaluates it. Returns exactly
// u < accept_threshold(x) (the accept probe, tests/test_gpu_math.py, checks 2^30 pairs).
__device__ __forceinline__ bool accept_u(float u, double x) {
    if (x >= 0.0) return u < 1.0f;
    if (x < -24.0) return false;
    const float e = __builtin_amdgcn_exp2f((float)x * 1.44269504f);
    if (u < e * 0.9999f) return true;
    if (u > e * 1.0001f) return false;
    return u < fminf(1.0f, (float)exp_ool(x));
}

// Accept's decision with the proposal's exact total `star` and the current total known only as
// the interval `cur` (after a proposal accepted on the bound): the threshold min(1, (float)exp(
// beta (star - cur))) does not increase with cur (the double difference of two floats is
// exact), so the decision is certain when u lies on one side of the thresholds at both ends --
// one float ulp apart from them, for the rounding of exp; 1 and 0 are exact. Then no exact pass
// of the current configuration is needed: BOUND_REJECT, BOUND_ACCEPT or BOUND_OPEN.
__device__ __forceinline__ int decide_exact_star(float star, CostIv cur, float u, double beta) {
    const float th_max = accept_threshold(beta * ((double)star - (double)cur.lo));
    const float th_min = accept_threshold(beta * ((double)star - (double)cur.hi));
    // (the next float up, for the non-negative finite u and thresholds)
    auto up = [](float v) { return __uint_as_float(__float_as_uint(v) + 1u); };
    int d = BOUND_OPEN;
    if (th_max == 0.0f ? u > 0.0f : u > up(th_max))
        d = BOUND_REJECT;
    else if (th_min == 1.0f ? u < 1.0f : up(u) < th_min)
        d = BOUND_ACCEPT;
    return __builtin_amdgcn_readfirstlane(d);
}

template <class Rng>
__device__ __forceinline__ bool accept(Rng& rng, float star, float cur) {
    const float u = rng.uniform();
    return u < accept_threshold(kBeta * ((double)star - (double)cur));
}

// The same at inverse temperature beta (parallel tempering; beta = kBeta is Accept itself).
template <class Rng>
__device__ __forceinline__ bool accept_at(Rng& rng, float star, float cur, double beta) {
    const float u = rng.uniform();
    return u < accept_threshold(beta * ((double)star - (double)cur));
}

}  // namespace mh
