/*
 * transport.hip — MI355X (gfx950) photon-packet transport kernels.
 *
 * A Monte-Carlo time step is processed in "generations".  Generation 0 =
 * the step's sources: census packets of the previous step
 * (src/imcfield2d.f:57-144), volume packets (src/imcvol2d_para.f:90-414) and
 * surface packets (src/imcsurf2d_para.f:228-534); generation g+1 = the
 * split2/split3 scatter secondaries of the collisions of generation g
 * (src/imctrk2d.f:580-684).  Three kernels:
 *
 *   c2d_source_kernel     samples the generation-0 volume/surface sources
 *                         into the packet store (PktSoA, one lane per packet);
 *   c2d_scatter_kernel    samples compb2d for every split2/split3 copy of the
 *                         generation's collision records, deposits the
 *                         energy change, and writes the secondaries to the
 *                         packet store (or a third-split record to q3);
 *   c2d_transport_kernel  the reference's recursive depth-first tracker
 *                         (src/imctrk2d.f:8-708) as a persistent per-lane
 *                         state machine: lane idle -> fetch a packet
 *                         (wave-aggregated, chunked atomic) -> split1 probe
 *                         copies, one packet-step per loop iteration ->
 *                         recombined unscattered copy (imctrk2d(0)) -> next.
 *
 * Keeping the rejection samplers out of the tracking loop keeps its register
 * footprint (and so its occupancy) at what one packet-step needs.  Packet
 * state never leaves registers between packet-steps; HBM sees only the
 * packet records, the census/event/collision appends (wave-ballot
 * compaction: one atomic per wave) and the tally flush.  Cell tallies
 * (edep, prdep, ecens, npcen) and escape tallies (fout, edout, erlk*) are
 * privatised per workgroup in LDS and flushed once with atomics.  Every
 * packet draws from its own Philox stream keyed by lineage (c2d_rng.h), so
 * a history does not depend on which lane/GPU/generation tracks it.
 *
 * Built twice (see Makefile): C2D_VARIANT=0 "exact" (comtot by the full
 * 199-term sum, -ffp-contract=off: bit-identical to the oracle's lineage
 * mode) and C2D_VARIANT=1 "fast" (comtot from the per-step cubic table,
 * cos(phi) carried between packet-steps, reciprocal-based division; also
 * -ffp-contract=off: contraction measured -3.3x).
 */
#include <hip/hip_runtime.h>

/* C2D_FAST_MDIV (fast build): the divisions inside c2d_math.h's log / exp /
 * acos series as a * (1/b) with the reciprocal from v_rcp_f64 and two Newton
 * steps (~1 ulp; the exact build keeps the IEEE quotient of the oracle) */
#ifndef C2D_FAST_MDIV
#define C2D_FAST_MDIV 1
#endif
#if defined(C2D_VARIANT) && C2D_VARIANT == 1 && C2D_FAST_MDIV
__device__ __forceinline__ double c2d_mdiv_rcp(double a, double b) {
  double y = __builtin_amdgcn_rcp(b);
  y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
  y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
  return a * y;
}
#define C2D_MDIV(a, b) c2d_mdiv_rcp((a), (b))
#endif
/* C2D_FAST_FMA (fast build): the Horner steps of those series (and of the
 * point loop's -log(1-x) series) as fused multiply-adds.  Off: gfx950's
 * v_fmac_f64 takes the addend in the destination VGPR, so each f64
 * coefficient costs two v_mov_b32 instead of two s_mov_b32 (+83 VALU
 * instructions in the bundle kernel, -117 in all) */
#ifndef C2D_FAST_FMA
#define C2D_FAST_FMA 0
#endif
#if defined(C2D_VARIANT) && C2D_VARIANT == 1 && C2D_FAST_FMA
#define C2D_MADD(a, b, c) __builtin_fma((a), (b), (c))
#endif

#include "c2d_device.hpp"
#include "c2d_math.h"
#include "c2d_rng.h"

#ifndef C2D_VARIANT
#define C2D_VARIANT 0
#endif
#if C2D_VARIANT == 0
#define C2D_SFX(x) x##_exact
#define C2D_TABLE_COMTOT 0
#else
#define C2D_SFX(x) x##_fast
#define C2D_TABLE_COMTOT 1
#endif

/* occupancy target of the transport kernel (waves per SIMD; 0 = compiler's
 * choice for BLOCK-thread groups, i.e. up to 256 VGPRs) */
#ifndef C2D_WAVES_PER_EU
#define C2D_WAVES_PER_EU 0
#endif
#if C2D_WAVES_PER_EU > 0
#define C2D_TR_ATTR __attribute__((amdgpu_waves_per_eu(C2D_WAVES_PER_EU)))
#else
#define C2D_TR_ATTR
#endif

namespace c2d {
/* the transport kernel's dynamic LDS: Geo image | cell tallies | escape tallies */
extern __shared__ double c2d_tr_lds[];
namespace {

constexpr double PI_REF = 3.1415926536;        /* general.pa:24 */
constexpr double C_LIGHT = 2.9979245620e10;    /* general.pa:25 */
constexpr double RAD_CP = 3.333564097e-11;     /* general.pa:23 */
constexpr double EMASSKEV = 5.11e2;
constexpr double SIGTHOM = 6.6516e-25;
constexpr int BLOCK = C2D_TR_BLOCK;   /* transport and bundle kernels */
constexpr int SBLOCK = 256;       /* scatter kernel */
/* source kernel: its LDS (the Geo image and the volume prefix, ~26 KB) per
 * workgroup limits a CU to 6 of them; 512 threads make that 8 waves per SIMD */
#ifndef C2D_SRC_BLOCK
#define C2D_SRC_BLOCK 512
#endif
constexpr int SRCBLOCK = C2D_SRC_BLOCK;
/* generation-0 items a wave takes per fetch (one returning atomic on a work
 * shard counter: 64 -> 256 -> 1024 items, +6 %, +2 %) */
#ifndef C2D_WORK_CHUNK
#define C2D_WORK_CHUNK C2D_CCHUNK
#endif
constexpr long long CHUNK = C2D_WORK_CHUNK;
/* fast build: -log(1-x) of the survivors' absorption points by its series
 * below 1e-2 (0: always the log, -3 %) */
#ifndef C2D_PT_SERIES
#define C2D_PT_SERIES 1
#endif
/* fast build: the survivors' absorption points in f32 (C2D_PT_F32=1; 0:
 * f64).  They only weight prdep (delpr = deleabs * wmustar * c,
 * imctrk2d.f:454-462: radiation pressure, read by no other part of the
 * reference); f32 keeps wmustar to ~1e-7, far inside the fast build's 1e-3
 * tally tolerance */
#ifndef C2D_PT_F32
#define C2D_PT_F32 1
#endif
/* fast build: the probe bundle's optical depth to its next collision,
 * tau = -log(u)/n, in f32 (C2D_TAU_F32=1; 0: the f64 log) to ~2e-7 relative
 * for every u (tau_log_f32).  tau only decides where the exponential
 * collision process puts the next collision, so that error leaves the
 * process's statistics unchanged.  In an optically thin medium a collision
 * needs u within ~1e-5 of 1: there (float)u would keep only 1-u to 6e-8
 * absolute (1e-3 relative in tau, and tau = 0 for u > 1 - 2^-25), so the
 * tail is taken from the complement 1 - u, exact in f64 */
#ifndef C2D_TAU_F32
#define C2D_TAU_F32 1
#endif
/* the census stream (records read once at a source's start, written once at
 * its census; the source kernel's volume records likewise) as non-temporal
 * accesses (C2D_CENS_NT=1, default): they need not stay in the XCD's 4 MB L2
 * beside the cell tables (comtot 4.4 MB + kappa 0.9 MB on C3), which every
 * flight step gathers.  C3 generation 0: 112.4 -> 106.7 ms (profiles/r09d,
 * r09e: two A/B pairs each, same histories) */
#ifndef C2D_CENS_NT
#define C2D_CENS_NT 1
#endif
/* the escape-event records likewise (C2D_EV_NT=1; measured neutral, r09e) */
#ifndef C2D_EV_NT
#define C2D_EV_NT 0
#endif
#define EV_ST(p, v) __builtin_nontemporal_store((double)(v), (C2D_GLOBAL double*)(p))
#if C2D_CENS_NT
#define CENS_ST2 cst2_nt
#define CENS_ST4 cst4_nt
#define CENS_LD2 cld2_nt
#define CENS_LD4 cld4_nt
#else
#define CENS_ST2 cst2
#define CENS_ST4 cst4
#define CENS_LD2 cld2
#define CENS_LD4 cld4
#endif
/* fast build: the comtot table coordinate ln(xnu) of a source with
 * v_log_f32 (C2D_LNX_F32=1).  An absolute error of ~1e-7 in ln(xnu) moves
 * the cubic interpolation point by 4e-6 of a table step (ln 1e25 / 2047),
 * ~1e-7 relative in comtot: the table's own interpolation error */
#ifndef C2D_LNX_F32
#define C2D_LNX_F32 1
#endif
#if C2D_TABLE_COMTOT && C2D_TAU_F32
#define TAU_LOG(u) c2d_tau_log_f32(u)
#else
#define TAU_LOG(u) FLOG(u)
#endif

/* Fast build only (the exact build keeps the oracle's c2d_math and IEEE
 * division bit for bit):
 *   C2D_FAST_EXP  1: exp by the ROCm device library (branch-free, ~42 VALU
 *                 instead of fdlibm's ~99 with its branches and division);
 *                 2: fdlibm's general path without its branches (exp_neg);
 *   C2D_FAST_DIV  a / b for b finite and nonzero as a * (1/b), the reciprocal
 *                 from v_rcp_f64 and two Newton steps (~1 ulp);
 *   C2D_RSQ_NR    Newton steps after v_rsq_f64 in the survivors' point loop.
 * A/B on the C3 census (profiles/r03_microopt.txt): FAST_DIV +2 % (on),
 * FAST_EXP=1 -4 % (ocml's exp keeps more VGPRs live), RSQ_NR=1 +1 %
 * (within noise then; round 4, two A/B pairs on the steady-state census,
 * profiles/r05j: generation 0 126.5/126.6 vs 126.9/126.9 ms, now the
 * default: one Newton step after v_rsq_f64 leaves 4.1e-15 relative in the
 * absorption-point deposits, r05k).  On the
 * steady-state C3 census (profiles/r03k): FAST_EXP=2 +1 % (default),
 * C2D_FAST_MDIV +1.2 %. */
#ifndef C2D_FAST_EXP
#define C2D_FAST_EXP 2
#endif
#ifndef C2D_FAST_DIV
#define C2D_FAST_DIV 1
#endif
#ifndef C2D_RSQ_NR
#define C2D_RSQ_NR 1
#endif
/* C2D_FAST_LOG (fast build): log(x) for normal x > 0 by fdlibm's reduction
 * and polynomial with one of its two final forms for every x (c2d_log_pos
 * evaluates both and the |f| < 2^-20 form, then selects): < 1 ulp (host
 * check against logl over (0,1), (0.7,1), e^[-40,40] and 1 +- 5e-7) */
#ifndef C2D_FAST_LOG
#define C2D_FAST_LOG 1
#endif
#if C2D_TABLE_COMTOT && C2D_FAST_LOG
__device__ __forceinline__ double log_fast(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  int32_t hx = c2d_hi(x);
  int32_t k = (hx >> 20) - 1023;
  hx &= 0x000fffff;
  const int32_t i = (hx + 0x95f64) & 0x100000;
  x = c2d_with_hi(x, hx | (i ^ 0x3ff00000));
  k += (i >> 20);
  const double f = x - 1.0, dk = (double)k;
  const double s = C2D_MDIV(f, 2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}
#define FLOG(x) log_fast(x)
#else
#define FLOG(x) c2d_log_pos(x)
#endif
#if C2D_TABLE_COMTOT && C2D_FAST_EXP == 1
#define FEXP(x) exp(x)
#elif C2D_TABLE_COMTOT && C2D_FAST_EXP == 2
/* exp(x) for -100 < x <= 0 (every use: exp(-xabs) with xabs < 100) without
 * branches: fdlibm's general reduction x = k ln2 + r for every x.  Its
 * |x| < 1.5 ln2 special cases are this path with k = 0 / -1 (same hi, lo and
 * result), and 2^k never leaves the normal range, so the result equals
 * c2d_exp except that |x| < 2^-28 gives 1 + x + x^2/2 before rounding. */
__device__ __forceinline__ double exp_neg(double x) {
  const double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00,
               P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  const int32_t k = (int32_t)(invln2 * x - 0.5);
  const double t = (double)k;
  const double hi = x - t * ln2HI, lo = t * ln2LO;
  const double r = hi - lo;
  const double rr = r * r;
  const double c = r - rr * (P1 + rr * (P2 + rr * (P3 + rr * (P4 + rr * P5))));
  const double y = 1.0 - ((lo - C2D_MDIV(r * c, 2.0 - c)) - hi);
  return c2d_with_hi(y, (int32_t)((uint32_t)c2d_hi(y) + ((uint32_t)k << 20)));
}
#define FEXP(x) exp_neg(x)
#else
#define FEXP(x) c2d_exp(x)
#endif
#if C2D_TABLE_COMTOT && C2D_FAST_DIV
/* C2D_FAST_NR: Newton steps after the v_rcp_f64 / v_rsq_f64 estimates of
 * the bundle step's divisions and square roots (rcp_pos, fsqrt_nn).  The
 * estimates are good to 4.6e-8 / 5.2e-8 relative, one step to 2.2e-15 /
 * 4.1e-15 over 1e-6..1e6 (tests/test_gpu_rcp_precision.py, r05k); one step:
 * generation 0 126.2/126.3 -> 125.4/125.5 ms in two A/B pairs (r05k) */
#ifndef C2D_FAST_NR
#define C2D_FAST_NR 1
#endif
__device__ __forceinline__ double rcp_pos(double b) {
  double y = __builtin_amdgcn_rcp(b);
#pragma unroll
  for (int k = 0; k < C2D_FAST_NR; k++) y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
  return y;
}
#define FDIV_POS(a, b) ((a) * rcp_pos(b))
/* C2D_FAST_SQRT: the bundle step's square roots (distances, radii, |sin|)
 * as x * rsq(x) with two Newton steps on rsq (~1 ulp; max rel. error of the
 * same sequence in the point loop 2.6e-16 on the box) instead of the
 * correctly rounded ~17-instruction sequence; x floored at 1e-300 so a zero
 * radius gives a tiny one (the quotients by it are clamped, FDIV_NN) */
#ifndef C2D_FAST_SQRT
#define C2D_FAST_SQRT 1
#endif
#if C2D_FAST_SQRT
__device__ __forceinline__ double fsqrt_nn(double x) {
  x = fmax(x, 1.0e-300);
  const double h = 0.5 * x;
  double y = __builtin_amdgcn_rsq(x);
#pragma unroll
  for (int k = 0; k < C2D_FAST_NR; k++) y = y * __builtin_fma(-h, y * y, 1.5);
  return x * y;
}
#define FSQRT(x) fsqrt_nn(x)
#else
#define FSQRT(x) __builtin_sqrt(x)
#endif
/* b >= 0 that may be 0 (a radius): b floored at 1e-300, so a / 0 gives a
 * huge value of a's sign (clamped by the caller) and 0 / 0 gives 0 */
#define FDIV_NN(a, b) ((a) * rcp_pos(fmax((b), 1.0e-300)))
#else
#define FDIV_POS(a, b) ((a) / (b))
#define FDIV_NN(a, b) ((a) / (b))
#define FSQRT(x) __builtin_sqrt(x)
#endif

/* Fortran REAL literals promoted to double (src/imcvol2d_para.f:204,221,247,268,336) */
#define F32(x) ((double)(float)(x))

enum : int32_t { FL_CONT = 0, FL_END = 1, FL_COLLIDE = 2 };

struct Pkt {
  double xnu, wmu, phi, rpre, zpre, dcen, ew, wtmin;
#if C2D_TABLE_COMTOT
  double eta;         /* fast build: cos(phi) carried between packet-steps       */
  double tt;          /* comtot table abscissa fraction for xnu                   */
  int32_t tg;         /* comtot table index (0: outside the table, exact sum)     */
  int32_t esw;        /* Eta_switch (quadrant of phi), constant between events    */
#endif
  int32_t jph, kph, mode;
  uint32_t bins;      /* jgpsp | jgplc << 8 | jgpmu << 16 | kap << 24 (PktSoA layout): the
                         spectral bins (imcleak2d.f) and the kappa phase (H3) in one register */
  int32_t ie;         /* E_ph bin of xnu (imctrk2d.f:382-384), cached per xnu, in the low
                         16 bits; its E_field bin + 1 above them (0: not known yet) */
  uint64_t key;
  uint32_t sub;       /* lineage sub-stream: split1 copies of a source (c2d_rng.h) */
  uint32_t ctr;
  uint32_t nflight;   /* safety cap: a history that stops progressing is aborted */
  double cmfp;        /* C2D_TRK_2012_11: colmfp carried across cell boundaries
                         (src_20121113/imctrk2d.f:505,526-533); unused otherwise */
};

__device__ __forceinline__ int32_t JGPSP(const Pkt& p) { return (int32_t)(p.bins & 0xffu); }
__device__ __forceinline__ int32_t JGPLC(const Pkt& p) { return (int32_t)((p.bins >> 8) & 0xffu); }
__device__ __forceinline__ int32_t JGPMU(const Pkt& p) { return (int32_t)((p.bins >> 16) & 0xffu); }
__device__ __forceinline__ int32_t KAP(const Pkt& p) { return (int32_t)(p.bins >> 24); }
__device__ __forceinline__ uint32_t pack_bins(int32_t sp, int32_t lc, int32_t mu, int32_t kap) {
  return (uint32_t)sp | ((uint32_t)lc << 8) | ((uint32_t)mu << 16) | ((uint32_t)kap << 24);
}
__device__ __forceinline__ void set_bins(Pkt& p, int32_t sp, int32_t lc, int32_t mu) {
  p.bins = pack_bins(sp, lc, mu, KAP(p));
}

/* Safety caps (never reached by a valid history; they keep a malformed input
 * from hanging the GPU).  Hitting one counts C2D_CNT_ABORTED. */
constexpr uint32_t MAX_FLIGHTS = 1u << 20;
constexpr int MAX_REJECT = 1 << 20;

/* Counters: packet-steps in a register (one per step), the rarer events
 * as LDS atomics on a per-workgroup array, flushed once at the end. */
__shared__ uint32_t c2d_cnt_lds[C2D_NCOUNTERS];   /* the workgroup's event counters */
struct LaneCnt {
  uint32_t steps;
  uint32_t paths;     /* lane path-steps (C2D_CNT_PATHS_INT) */
};
#define LC_ADD(lc, which) atomicAdd(&c2d_cnt_lds[which], 1u)

/* Tally views.  Cell tallies edep|prdep|ecens|npcen (stride ncell) and
 * escape tallies fout|edout|erlki|erlko|erlku|erlkl have the same layout in
 * LDS and in the fused global buffer.  LDS addresses are formed from the
 * c2d_tr_lds symbol (offsets, not stored pointers) so the compiler emits ds_*
 * instructions instead of flat ones with a run-time address-space dispatch. */
struct Tal {
  const Geo* g;      /* LDS image of the grids */
  int cells_off;     /* offset of the privatised cell tallies in c2d_tr_lds (P.lds_cells) */
  int esc_off;       /* offset of the escape tallies in c2d_tr_lds */
};
#define T_FOUT(P, T) (c2d_tr_lds + (T).esc_off)
#define T_EDOUT(P, T) (T_FOUT(P, T) + (P).nmu * C2D_NPHOMAX)
#define T_ERLKI(P, T) (T_FOUT(P, T) + (P).nmu * (C2D_NPHOMAX + C2D_NPHLCMAX))
#define T_ERLKO(P, T) (T_ERLKI(P, T) + (P).nz)
#define T_ERLKU(P, T) (T_ERLKI(P, T) + 2 * (P).nz)
#define T_ERLKL(P, T) (T_ERLKI(P, T) + 2 * (P).nz + (P).nr)
enum : int { TC_EDEP = 0, TC_PRDEP = 1, TC_ECENS = 2, TC_NPCEN = 3 };
/* cell tallies edep|prdep|ecens|npcen: LDS when privatised, else the fused buffer */
__device__ __forceinline__ void cell_add(const KParams& P, const Tal& T, int which, int cell, double v) {
#ifdef C2D_ABLATE_CELL_TALLY            /* profiling ablation only (tools/build_sweep.sh) */
  if (v != 12345.0) return;
#endif
  if (P.lds_cells) atomicAdd(&c2d_tr_lds[T.cells_off + which * P.ncell + cell], v);
  else gadd(P.T + P.off.edep + which * P.ncell + cell, v);
}

/* Rare paths (census writes, escapes, collision records, source loads) read
 * their KParams fields through an opaque copy of the pointer: the loads
 * stay in those paths instead of being hoisted out of the lane loop, where
 * they would hold ~70 SGPRs for the whole launch and spill (C2D_COLD_RELOAD=0
 * restores the hoisted form). */
#ifndef C2D_COLD_RELOAD
#define C2D_COLD_RELOAD 0
#endif
/* C2D_COLD_CALL: the rare event paths (census write, escape) as real calls,
 * so their temporaries do not add to the lane loop's register pressure */
/* C2D_EARLY_LOADS (fast build): issue a step's table loads at its start */
#ifndef C2D_EARLY_LOADS
#define C2D_EARLY_LOADS 0
#endif
#ifndef C2D_COLD_CALL
#define C2D_COLD_CALL 0
#endif
#if C2D_COLD_CALL
#define C2D_COLD_FN __device__ __noinline__
#else
#define C2D_COLD_FN __device__ __forceinline__
#endif
__device__ __forceinline__ const KParams& cold(const KParams& P) {
#if C2D_COLD_RELOAD
  const KParams* q = &P;
  asm volatile("" : "+s"(q));
  return *q;
#else
  return P;
#endif
}

__device__ __forceinline__ const KParams& cold_always(const KParams& P) {
  const KParams* q = &P;
  asm volatile("" : "+s"(q));
  return *q;
}

/* Next draw of the packet's stream (every key change sets ctr = 0; a packet
 * loaded from a record resumes at the record's ctr). */
__device__ __forceinline__ double U(Pkt& p) {
  return c2d_draw_s(p.key, p.sub, p.ctr++);
}

__device__ __forceinline__ double clampd(double v, double lim) {
  if (v > lim) v = lim;
  if (v < -lim) v = -lim;
  return v;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

/* Wave-ballot compaction: the lanes executing this call reserve consecutive
 * slots of *counter with a single atomic. */
__device__ __forceinline__ unsigned long long wave_reserve(unsigned long long* counter) {
  unsigned long long mask = __ballot(1);
  uint32_t leader = (uint32_t)(__ffsll((long long)mask) - 1);
  uint32_t lane = lane_id();
  unsigned long long lt = (lane == 0) ? 0ull : (mask & ((~0ull) >> (64 - lane)));
  uint32_t rank = (uint32_t)__popcll(lt);
  unsigned long long base = 0;
  if (lane == leader)
    base = __hip_atomic_fetch_add((C2D_GLOBAL unsigned long long*)counter,
                                  (unsigned long long)__popcll(mask), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
  uint32_t lo = __builtin_amdgcn_readlane((uint32_t)base, leader);
  uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(base >> 32), leader);
  return (((unsigned long long)hi << 32) | lo) + rank;
}

/* ------------------------------------------------------------------ */
/* comtot (src/comtot2d.f:1-334, icoms=6 :219-247), intg_v :337, dilog :356 */
/* ------------------------------------------------------------------ */
__device__ double dilog(double x) {
  const double C[21] = {0,
      0.42996693560813697, 0.40975987533077105, -0.01858843665014592,
      0.00145751084062268, -0.00014304184442340, 0.1588415541880e-4,
      -0.190784959387e-5, 0.024195180854e-5, -0.003193341274e-5,
      0.000434545063e-5, -0.000060578480e-5, 0.000008612098e-5,
      -0.000001244332e-5, 0.000000182256e-5, -0.000000027007e-5,
      0.000000004042e-5, -0.000000000610e-5, 0.000000000093e-5,
      -0.000000000014e-5, 0.000000000002e-5};
  const double HF = 0.5, PI2 = PI_REF * PI_REF, PI3 = PI2 / 3, PI6 = PI2 / 6,
               PI12 = PI2 / 12;
  double T, H, Y, S, A, ALFA, B1, B2, B0 = 0.0;
  if (x == 1) {
    H = PI6;
  } else if (x == -1) {
    H = -PI12;
  } else {
    T = -x;
    if (T <= -2) {
      Y = -1 / (1 + T);
      S = 1;
      B1 = c2d_log(-T);
      B2 = c2d_log(1 + 1 / T);
      A = -PI3 + HF * (B1 * B1 - B2 * B2);
    } else if (T < -1) {
      Y = -1 - T;
      S = -1;
      A = c2d_log(-T);
      A = -PI6 + A * (A + c2d_log(1 + 1 / T));
    } else if (T <= -0.5) {
      Y = -(1 + T) / T;
      S = 1;
      A = c2d_log(-T);
      A = -PI6 + A * (-HF * A + c2d_log(1 + T));
    } else if (T < 0) {
      Y = -T / (1 + T);
      S = -1;
      B1 = c2d_log(1 + T);
      A = HF * B1 * B1;
    } else if (T <= 1) {
      Y = T;
      S = 1;
      A = 0;
    } else {
      Y = 1 / T;
      S = -1;
      B1 = c2d_log(T);
      A = PI6 + HF * B1 * B1;
    }
    H = Y + Y - 1;
    ALFA = H + H;
    B1 = 0;
    B2 = 0;
#pragma unroll
    for (int i = 20; i >= 1; i--) {
      B0 = C[i] + ALFA * B1 - B2;
      B2 = B1;
      B1 = B0;
    }
    H = -(S * (B0 - H * B2) + A);
  }
  return H;
}

__device__ __forceinline__ double intg_v(double x) {
  double i1 = -x / 2.0 + 0.5 / (1.0 + x);
  double i2 = 4.0 * dilog(-x);
  double i3 = (9.0 + x + 8.0 / x) * c2d_log(1.0 + x);
  return i1 + i2 + i3;
}

/* cross section for one Lorentz-factor bin i (1-based): sigma_E(i, x) */
__device__ __forceinline__ double sigma_E_bin(double gnti, double x) {
  double gamma0 = gnti + 1.0;
  double betta = __builtin_sqrt(1.0 - 1.0 / (gamma0 * gamma0));
  if (x * gamma0 * (1 + betta) < 1.0e-2) return SIGTHOM * (1.0 - 2.0 * x * gamma0);
  return 9.375e-2 * SIGTHOM / (gamma0 * gamma0) / betta / (x * x) *
         (intg_v(2 * gamma0 * (1 + betta) * x) - intg_v(2 * gamma0 * (1 - betta) * x));
}

__device__ __noinline__ double comtot_exact(const KParams& P, int cell, double xnuc) {
  const double* fnt = P.f_nt + (int64_t)cell * C2D_NUM_NT;
  double cosig = 0.0, x = xnuc / EMASSKEV;
  for (int i = 1; i <= C2D_NUM_NT - 1; i++) {
    double gi = P.gnt[i - 1], gi1 = P.gnt[i];
    double sE = sigma_E_bin(gi, x);
    cosig = cosig + sE * fnt[i - 1] * (gi1 - gi);
  }
  if (cosig < 1.0e-40) return 1.0e-40;
  return P.n_e[cell] * cosig;
}

#if C2D_TABLE_COMTOT
/* cubic Lagrange interpolation of the per-step table at the packet's cached
 * abscissa (tg, tt); tg == 0 means xnu lies outside the table: exact sum. */
__device__ __forceinline__ double comtot_interp(double y0, double y1, double y2, double y3,
                                                double ne, double t) {
  const double tm1 = t - 1.0, tm2 = t - 2.0, tp1 = t + 1.0;
  const double cosig = -(t * tm1 * tm2) * (1.0 / 6.0) * y0 + (tp1 * tm1 * tm2) * 0.5 * y1 -
                       (tp1 * t * tm2) * 0.5 * y2 + (tp1 * t * tm1) * (1.0 / 6.0) * y3;
  if (cosig < 1.0e-40) return 1.0e-40;
  return ne * cosig;
}
__device__ __forceinline__ double comtot_table(const KParams& P, int cell, const double xnu,
                                               const int tg, const double t) {
  if (tg == 0) return comtot_exact(P, cell, xnu);
  const double* tb = P.comtab + (int64_t)cell * C2D_COMTAB_N + (tg - 1);
  return comtot_interp(gld(tb), gld(tb + 1), gld(tb + 2), gld(tb + 3), gld(P.n_e + cell), t);
}
#endif

/* ------------------------------------------------------------------ */
/* binning (src/compb_2d.f:249-302, src/imcleak2d.f:329-405)            */
/* ------------------------------------------------------------------ */
__device__ __forceinline__ int bin_sp(const Geo* g, int nphtotal, double xnu, double fbot,
                                      double ftop, int top_value) {
  int jbot = 1, jtop = nphtotal + 1, jmid;
  double hubot = fbot * g->hu[1];
  double hutop = ftop * g->hu[jtop];
  if (xnu >= hutop) return top_value;
  if (xnu <= hubot) return 0;
  for (;;) {
    jmid = (jbot + jtop) / 2;
    if (jmid == jbot) break;
    if (xnu == g->hu[jmid]) break;
    if (xnu < g->hu[jmid]) jtop = jmid;
    else jbot = jmid;
  }
  return jmid;
}
__device__ __forceinline__ int bin_lc(const Geo* g, int nph_lc, double xnu) {
  for (int m = 1; m <= nph_lc; m++)
    if (xnu > g->Elcmin[m] && xnu <= g->Elcmax[m]) return m;
  return 0;
}
__device__ __forceinline__ int bin_mu(const Geo* g, int nmu, double wmu) {
  for (int n = 1; n <= nmu; n++)
    if (wmu <= g->mu[n]) return n;
  return nmu;
}
/* first i in 1..n-1 with x < E[i+1], else n (the reference's linear scans
 * imctrk2d.f:382-384 and :547-549), by bisection on a monotone grid */
__device__ __forceinline__ int grid_index(const double* E, int n, double x) {
  int lo = 1, hi = n;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (x < E[mid + 1]) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}
/* grid_index through the Geo bucket table (c2d_device.hpp): the same bin,
 * one LDS read and an upward scan of <= 2 bins instead of a 9-deep chain of
 * dependent LDS reads.  x > 0. */
__device__ __forceinline__ int grid_lookup(const double* E, int n, const int16_t* start, int32_t k0,
                                           double x) {
  int b = (int)(c2d_bits(x) >> 48) - k0;
  b = b < 0 ? 0 : (b > C2D_IDX_BUCKETS - 1 ? C2D_IDX_BUCKETS - 1 : b);
  int i = start[b];
  while (i < n && !(x < E[i + 1])) i++;
  return i;
}
/* `i=0; do i=i+1 while (cdf(i) < rnum .and. i < n)` (imcvol2d_para.f:170-172) */
__device__ __forceinline__ int cdf_index(const double* cdf /*0-based*/, int n, double rnum,
                                         int linear, const uint16_t* guide = nullptr) {
  if (linear) {
    int i = 0;
    do { i = i + 1; } while (cdf[i - 1] < rnum && i < n);
    return i;
  }
  int lo = 1, hi = n;   /* smallest i with cdf(i) >= rnum, capped at n */
  if (guide) {
    /* the answer lies in [guide[q], guide[q+1]] for q = floor(rnum G)
     * (rnum G is exact, G a power of two): the same index in ~2 probes
     * instead of ~9 dependent loads */
    int q = (int)(rnum * (double)C2D_CDF_GUIDE);
    q = q < 0 ? 0 : (q > C2D_CDF_GUIDE - 1 ? C2D_CDF_GUIDE - 1 : q);
    lo = guide[q];
    hi = guide[q + 1];
  }
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (cdf[mid - 1] < rnum) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

/* ------------------------------------------------------------------ */
/* nth2d (src/nontherm2d.f:159-183) + compb2d (src/compb_2d.f:1-318)    */
/* ------------------------------------------------------------------ */
/* compb2d in three parts, so that its first rejection loop (electron +
 * Klein-Nishina acceptance, compb_2d.f:59-93) can run wave-parallel when it
 * is long (acceptance ~1e-5 for photons deep in the KN regime):
 *   kn_loop   a lane's own iterations, at most `cap` of them;
 *   kn_coop   wave-uniform: every lane left without an acceptance is resolved
 *             by the whole wave, 64 iterations per round;
 *   compb2d_b the rest of the scatter (:98-307).
 * Iteration j of the first loop draws its five uniforms from positions
 * ctrA + 5j .. ctrA + 5j + 4 of the packet's stream (ctrA: the counter at
 * the loop's start; an iteration that skips at znue < 1e-10 leaves its fifth
 * unused), so iterations are independent; the oracle's lineage mode draws
 * the same (oracle/c2d_oracle.c compb2d).
 * TALLY = +1: the nelectron samples and counters are added; -1: subtracted
 * again (a speculative split3 attempt beyond the first success,
 * c2d_scatter_hard_kernel). */
#define CB_CNT(w) do { if (TALLY > 0) atomicAdd(&c2d_cnt_lds[w], 1u); else atomicSub(&c2d_cnt_lds[w], 1u); } while (0)

struct KnState {
  double gamm, betb, omeg, znue;
  int i;            /* electron bin (i_gam) */
  uint32_t ctrA;    /* the packet's counter at the loop's start */
  int j;            /* iterations run (the next one to run) */
};

/* iteration j of the first loop; true if accepted */
__device__ __forceinline__ bool kn_iter(const KParams& P, Pkt& p, uint32_t ctrA, int j, double znu,
                                        KnState& st) {
  const double lim = 9.9999999e-1;
  const int cell = (p.jph - 1) * P.nr + (p.kph - 1);
  const double* Pc = P.Pnt + (int64_t)cell * C2D_NUM_NT;
  p.ctr = ctrA + 5u * (uint32_t)j;
  /* nth2d (nontherm2d.f:159-183) */
  double rnum = U(p);
  rnum = (double)(int32_t)(rnum * 1.0e6) / 1.0e6 + 1.0e-6 * U(p);
  int i = 2;
  {   /* first i in 2..200 with Pnt(i) > rnum, else 201 (bisection on the CDF) */
    int lo = 2, hi = C2D_NUM_NT + 1;
    while (lo < hi) {
      int mid = (lo + hi) >> 1;
      if (Pc[mid - 1] > rnum) hi = mid;
      else lo = mid + 1;
    }
    i = lo > C2D_NUM_NT ? C2D_NUM_NT : lo;   /* Pnt(200) = 1 > rnum in valid input */
  }
  const double gamm = __builtin_sqrt(P.gnt[i - 1] * P.gnt[i - 2]) + 1.0;
  const double betb = __builtin_sqrt(1.0 - 1.0 / (gamm * gamm));
  double omeg = 2.0 * U(p) - 1.0;
  omeg = clampd(omeg, lim);
  const double tl = U(p);
  const double tr = 0.5 * (1.0 - betb * omeg);
  if (tl > tr) omeg = -omeg;
  omeg = clampd(omeg, lim);
  const double znue = (1.0 - betb * omeg) * znu * gamm;
  st.i = i; st.gamm = gamm; st.betb = betb; st.omeg = omeg; st.znue = znue;
  if (znue < 1.0e-10) return false;
  double xknot;
  if (znue <= 1.0e-2) {
    xknot = 1.0 - znue * (2.0 - znue * (5.2 - znue * (13.3 - 1.144e3 * znue / 3.5e1)));
  } else {
    double znue3 = znue * znue * znue;
    double betz = 1.0 + 2.0 * znue;
    double gamz = znue * (znue - 2.0) - 2.0;
    double xxx = 4.0 * znue + 2.0 * znue3 * (1.0 + znue) / (betz * betz) + gamz * c2d_log(betz);
    xknot = 3.75e-1 * xxx / znue3;
  }
  p.ctr = ctrA + 5u * (uint32_t)j + 4u;
  return !(U(p) > xknot);
}

/* a lane's own iterations of the first loop, at most cap; true when one was
 * accepted (p.ctr then follows it) */
template <int TALLY = 1>
__device__ __forceinline__ bool kn_loop(const KParams& P, double* nel, Pkt& p, KnState& st, int cap) {
  CB_CNT(C2D_CNT_COMPB);
  st.ctrA = p.ctr;
  st.j = 0;
  const double znu = p.xnu / EMASSKEV;
  for (; st.j < cap; st.j++) {
    const bool ok = kn_iter(P, p, st.ctrA, st.j, znu, st);
    atomicAdd(&nel[st.i], (double)TALLY);
    if (ok) {
      st.j++;
      p.ctr = st.ctrA + 5u * (uint32_t)st.j;
      return true;
    }
  }
  return false;
}

__device__ __forceinline__ double rl_d(double v, uint32_t l) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

/* wave-uniform: every lane with `need` (its kn_loop ran out of iterations)
 * is resolved by the whole wave, lane after lane, 64 iterations per round;
 * iteration MAX_REJECT - 1 ends a loop the reference would not end
 * (C2D_CNT_ABORTED, as the sequential guard) */
template <int TALLY = 1>
__device__ __forceinline__ void kn_coop(const KParams& P, double* nel, Pkt& p, KnState& st, bool& need) {
  const uint32_t lane = lane_id();
  for (;;) {
    const unsigned long long m = __ballot(need);
    if (m == 0ull) break;
    const uint32_t L = (uint32_t)(__ffsll((long long)m) - 1);
    /* the owner's packet as the iterations read it */
    Pkt q;
    /* readlane returns int: through uint32_t, so the low word is not sign-extended */
    q.key = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)p.key, L) |
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(p.key >> 32), L) << 32);
    q.sub = __builtin_amdgcn_readlane(p.sub, L);
    q.jph = __builtin_amdgcn_readlane(p.jph, L);
    q.kph = __builtin_amdgcn_readlane(p.kph, L);
    const double znu = rl_d(p.xnu, L) / EMASSKEV;
    const uint32_t ctrA = __builtin_amdgcn_readlane(st.ctrA, L);
    int j0 = __builtin_amdgcn_readlane(st.j, L);
    for (;;) {
      const int j = j0 + (int)lane;
      KnState t;
      t.i = 0; t.gamm = t.betb = t.omeg = t.znue = 0.0;
      const bool live = j < MAX_REJECT;
      const bool acc = live && kn_iter(P, q, ctrA, j, znu, t);
      const bool ok = acc || j == MAX_REJECT - 1;
      const unsigned long long ma = __ballot(ok);
      const uint32_t jf = ma ? (uint32_t)(__ffsll((long long)ma) - 1) : 64u;
      if (live && lane <= jf) atomicAdd(&nel[t.i], (double)TALLY);
      if (ma) {
        const bool abort = __builtin_amdgcn_readlane((uint32_t)(!acc), jf) != 0u;
        const double gamm = rl_d(t.gamm, jf), betb = rl_d(t.betb, jf);
        const double omeg = rl_d(t.omeg, jf), znue = rl_d(t.znue, jf);
        const int ii = __builtin_amdgcn_readlane(t.i, jf);
        if (lane == L) {
          st.gamm = gamm; st.betb = betb; st.omeg = omeg; st.znue = znue; st.i = ii;
          st.j = j0 + (int)jf + 1;
          p.ctr = ctrA + 5u * (uint32_t)st.j;
          need = false;
          if (abort) CB_CNT(C2D_CNT_ABORTED);
        }
        break;
      }
      j0 += 64;
    }
  }
}

/* the rest of compb2d (:98-307) from the accepted electron */
template <int TALLY = 1>
__device__ __forceinline__ int compb2d_b(const KParams& P, const Geo* g, Pkt& p, const KnState& st) {
  const double fuzz = 1.0e-10, lim = 9.9999999e-1;
  const double znu = p.xnu / EMASSKEV;
  const double gamm = st.gamm, betb = st.betb, omeg = st.omeg, znue = st.znue;
  double sz, games, phat, znues, wa, wb, swa, tr;
  int guard = st.j;
  const double betz = 1.0 + 2.0 * znue;
  for (;;) {
    if (++guard > 2 * MAX_REJECT) { CB_CNT(C2D_CNT_ABORTED); break; }
    sz = (1.0 + 2.0 * znue * U(p)) / betz;
    games = 1.0 + (1.0 - 1.0 / sz) / znue;
    if ((1.0 - games * games) < 0.0) continue;
    tr = games * games - 1.0 + sz + 1.0 / sz;
    phat = betz + 1.0 / betz;
    if (U(p) * phat > tr) continue;
    break;
  }
  znues = znue * sz;
  for (;;) {
    if (++guard > 3 * MAX_REJECT) { CB_CNT(C2D_CNT_ABORTED); break; }
    wa = U(p);
    wb = 2.0 * U(p) - 1.0;
    swa = wa * wa + wb * wb;
    if (swa >= 1.0 || swa <= 1.0e-20) continue;
    break;
  }
  double cazes = (wa * wa - wb * wb) / swa;
  double omege = clampd((omeg - betb) / (1.0 - betb * omeg), lim);
  double omeges = games * omege +
                  cazes * __builtin_sqrt((1.0 - omege * omege + fuzz) * (1.0 - games * games));
  omeges = clampd(omeges, lim);
  double znus = (1.0 + betb * omeges) * gamm * znues;
  double gams = clampd(1.0 - (znue - znues) / (znu * znus), lim);
  for (;;) {
    if (++guard > 4 * MAX_REJECT) { CB_CNT(C2D_CNT_ABORTED); break; }
    wa = U(p);
    wb = 2.0 * U(p) - 1.0;
    swa = wa * wa + wb * wb;
    if (swa >= 1.0 || swa <= 1.0e-20) continue;
    break;
  }
  double cazs = clampd((wa * wa - wb * wb) / swa, lim);
  double wmus = p.wmu * gams +
                cazs * __builtin_sqrt((1.0 - gams * gams) * (1.0 - p.wmu * p.wmu + fuzz));
  wmus = clampd(wmus, lim);
  double xnus = znus * EMASSKEV;
  double cosdphi = clampd((gams - p.wmu * wmus) /
                              __builtin_sqrt((1.0 - p.wmu * p.wmu) * (1.0 - wmus * wmus)),
                          lim);
  double dphi = c2d_acos(cosdphi);
  double phis = p.phi + dphi;
  set_bins(p, bin_sp(g, P.nphtotal, xnus, 1.000001, 0.999999, 0), bin_lc(g, P.nph_lc, xnus),
           bin_mu(g, P.nmu, wmus));
  p.ew = p.ew * xnus / p.xnu;
  p.xnu = xnus;
  p.wmu = wmus;
  p.phi = phis;
  return st.i;
}

/* wave-uniform compb2d (imctrk2d.f's `call compb2d`, compb_2d.f:1-318): every
 * lane calls it; lanes with run = false take no part but the wave's
 * cooperation.  Returns i_gam for running lanes. */
template <int TALLY = 1>
__device__ __forceinline__ int compb2d_w(const KParams& P, const Geo* g, double* nel, Pkt& p, bool run,
                                          int kn_cap) {
  KnState st;
  st.i = 0; st.j = 0; st.ctrA = 0;
  bool need = false;
  /* kn_coop needs a live iteration left (it ends at MAX_REJECT - 1) */
  if (run) need = !kn_loop<TALLY>(P, nel, p, st, kn_cap < MAX_REJECT - 1 ? kn_cap : MAX_REJECT - 1);
  kn_coop<TALLY>(P, nel, p, st, need);
  int i_gam = 0;
  if (run) i_gam = compb2d_b<TALLY>(P, g, p, st);
  return i_gam;
}

/* ------------------------------------------------------------------ */
/* escapes (src/imcleak2d.f:2-320, cr_sent = 0)                          */
/* ------------------------------------------------------------------ */
__device__ __forceinline__ void push_event(const KParams& P0, double tb, const Pkt& p, LaneCnt& lc) {
  const KParams& P = cold(P0);
  const unsigned sh = blockIdx.x % C2D_EV_SHARDS;
  const unsigned long long slot = wave_reserve(P.n_ev_sh + sh * C2D_EV_SHARD_STRIDE);
  if (slot < (unsigned long long)P.cap_ev_sh) {
    double* e = P.ev + ((int64_t)sh * P.cap_ev_sh + (int64_t)slot) * C2D_EVENT_WORDS;
#if C2D_EV_NT
    EV_ST(e, tb); EV_ST(e + 1, p.xnu); EV_ST(e + 2, p.ew); EV_ST(e + 3, p.rpre); EV_ST(e + 4, p.zpre);
    EV_ST(e + 5, p.wmu); EV_ST(e + 6, p.phi);
#else
    gst(e, tb); gst(e + 1, p.xnu); gst(e + 2, p.ew); gst(e + 3, p.rpre); gst(e + 4, p.zpre);
    gst(e + 5, p.wmu); gst(e + 6, p.phi);
#endif
  } else {
    gor(P.err, ERR_EVENT);
  }
  LC_ADD(lc, C2D_CNT_EVENTS);
}

__device__ __forceinline__ void escape_tally(const KParams& P0, const Tal& T, const Pkt& p) {
  const KParams& P = cold(P0);
  const int32_t jgpsp = JGPSP(p), jgplc = JGPLC(p), jgpmu = JGPMU(p);
  if (jgplc > 0) atomicAdd(&T_EDOUT(P, T)[(jgpmu - 1) * C2D_NPHLCMAX + (jgplc - 1)], FDIV_POS(p.ew, P.dt));
  if (jgpsp > 0 && P.spec_switch == 0)
    atomicAdd(&T_FOUT(P, T)[(jgpmu - 1) * C2D_NPHOMAX + (jgpsp - 1)], p.ew);
}

/* returns idead: 1 = left the system, 0 = continue (axis pass-through) */
C2D_COLD_FN int imcleak(const KParams& P0, const Tal& T, Pkt& p, LaneCnt& lc) {
  const KParams& P = cold(P0);
  if (p.kph == 0) {
    if (P.rmin > 1.0e-10) {
      atomicAdd(&T_ERLKI(P, T)[p.jph - 1], p.ew);
      LC_ADD(lc, C2D_CNT_ESCAPES);
      return 1;
    }
    p.phi = 1.0e-6;
    p.kph = 1;
    return 0;
  }
  LC_ADD(lc, C2D_CNT_ESCAPES);
  const double tb = P.time + P.dt - RAD_CP * p.dcen;   /* H4: fresh t_bound everywhere */
  if (p.jph <= 0) {
    if (P.tbbl[p.kph - 1] > 0.0) {
      gadd(&P.T[P.off.Ed_in + p.kph - 1], p.ew);
      atomicAdd(&T_ERLKL(P, T)[p.kph - 1], p.ew);
    }
    if (P.ncycle > 0) {
      push_event(P, tb, p, lc);
      escape_tally(P, T, p);
    }
    return 1;
  }
  if (p.jph != P.nz + 1) {
    atomicAdd(&T_ERLKO(P, T)[p.jph - 1], p.ew);
    if (P.ncycle > 0) {
      push_event(P, tb, p, lc);
      escape_tally(P, T, p);
    }
    return 1;
  }
  atomicAdd(&T_ERLKU(P, T)[p.kph - 1], p.ew);
  if (P.ncycle > 0 && p.wmu < F32(0.98)) {
    push_event(P, tb, p, lc);
    escape_tally(P, T, p);
  }
  return 1;
}

/* Census appends come from wave-private chunks of P.cens_chunk slots,
 * reserved with one atomic (a single address every wave appends to:
 * per-write reservations were the kernel's limiter).
 *   double-buffered: chunks of up to 1024 slots (host: at most 1/8 of the
 *     capacity over all waves; 256 -> 1024 was +1 %) cut from the output
 *     counter; after the step the host marks the unused tail of each wave
 *     slot's last chunk dead and its compaction closes them;
 *   chunked: C2D_CCHUNK-slot chunks, first from the wave's stack of chunks
 *     its finished census sources freed, then from the relist, then from the
 *     step's free pool; each is listed in out_list when taken.
 * In both, a wave slot's partly filled chunk carries over to the next launch
 * of the step (cstate). */
/* per wave of the workgroup, in LDS (updated by the lanes that write) */
__shared__ unsigned long long c2d_cch_base[C2D_TR_BLOCK / 64];
__shared__ uint32_t c2d_cch_used[C2D_TR_BLOCK / 64];
/* chunked census, bundle kernel: the census chunks each wave counts down
 * (chunk index in the input list, -1 free; sources not yet finished) and its
 * stack of freed chunks */
__shared__ int32_t c2d_ct_idx[C2D_TR_BLOCK / 64][C2D_CT_TRACK];
__shared__ uint32_t c2d_ct_rem[C2D_TR_BLOCK / 64][C2D_CT_TRACK];
__shared__ int32_t c2d_fs[C2D_TR_BLOCK / 64][C2D_CT_STACK];
__shared__ uint32_t c2d_fs_n[C2D_TR_BLOCK / 64];
static_assert(C2D_WORK_CHUNK == C2D_CCHUNK, "a work chunk must cover exactly one census chunk");

/* the next chunk of the wave (leader lane): its first slot, or cap_cout when
 * none is left (the writes then fail with ERR_CENSUS) */
C2D_COLD_FN unsigned long long census_new_chunk(const KParams& P0, int w) {
  const KParams& P = cold(P0);
  if (!P.clist)
    return __hip_atomic_fetch_add((C2D_GLOBAL unsigned long long*)P.n_cout, (unsigned long long)P.cens_chunk,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int32_t id = -1;
  const uint32_t ns = c2d_fs_n[w];
  if (ns > 0) {
    id = c2d_fs[w][ns - 1];
    c2d_fs_n[w] = ns - 1;
  } else {
    /* an entry reserved but not yet written reads -1: its chunk sits out the step */
    if (__hip_atomic_load((C2D_GLOBAL unsigned long long*)P.n_relist, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT) > __hip_atomic_load((C2D_GLOBAL unsigned long long*)
                                                                          P.relist_head, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_AGENT)) {
      const unsigned long long h = atomicAdd(P.relist_head, 1ull);
      if (h < gld(P.n_relist))
        id = __hip_atomic_load((C2D_GLOBAL int32_t*)(P.relist + h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (id < 0) {
      const unsigned long long h = atomicAdd(P.pool_head, 1ull);
      if (h < gld(P.pool_n)) id = gld(P.pool + h);
    }
  }
  if (id < 0) return (unsigned long long)P.cap_cout;
  gst(P.out_list + atomicAdd(P.n_out, 1ull), id);
  return (unsigned long long)id << C2D_CCHUNK_LOG;
}

__device__ __forceinline__ unsigned long long census_slot_chunk(const KParams& P0) {
  const KParams& P = cold(P0);
  const int w = (int)(threadIdx.x >> 6);
  const unsigned long long mask = __ballot(1);
  const uint32_t leader = (uint32_t)(__ffsll((long long)mask) - 1);
  const uint32_t lane = lane_id();
  const unsigned long long lt = (lane == 0) ? 0ull : (mask & ((~0ull) >> (64 - lane)));
  const uint32_t rank = (uint32_t)__popcll(lt), k = (uint32_t)__popcll(mask);
  const unsigned long long base = c2d_cch_base[w];
  const uint32_t used = c2d_cch_used[w];
  const uint32_t CENS_CHUNK = P.cens_chunk;
  const uint32_t rem = CENS_CHUNK - used;
  if (k <= rem) {
    if (lane == leader) c2d_cch_used[w] = used + k;
    return base + used + rank;
  }
  unsigned long long nb = 0;
  if (lane == leader) nb = census_new_chunk(P, w);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)nb, leader);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(nb >> 32), leader);
  nb = ((unsigned long long)hi << 32) | lo;
  if (lane == leader) { c2d_cch_base[w] = nb; c2d_cch_used[w] = k - rem; }
  return rank < rem ? base + used + rank : nb + (rank - rem);
}

/* A wave slot's partly filled chunk carries over from launch to launch of
 * the step (cstate), so each wave slot leaves at most one per step: the
 * host closes them after the last generation (capi.cpp). */
__device__ __forceinline__ void census_chunk_load(const KParams& P0, int w, uint32_t lane) {
  const KParams& P = cold(P0);
  if (lane != 0) return;
  c2d_cch_base[w] = 0ull;
  c2d_cch_used[w] = P.cens_chunk;
  c2d_fs_n[w] = 0u;
  for (int e = 0; e < C2D_CT_TRACK; e++) c2d_ct_idx[w][e] = -1;
  const int64_t ws = (int64_t)blockIdx.x * (C2D_TR_BLOCK / 64) + w;
  const int64_t base = gld(P.cstate + 2 * ws);
  if (base >= 0) {
    c2d_cch_base[w] = (unsigned long long)base;
    c2d_cch_used[w] = (uint32_t)gld(P.cstate + 2 * ws + 1);
  }
}

/* a freed chunk the wave cannot keep goes to the relist */
__device__ __forceinline__ void census_relist(const KParams& P, int32_t id) {
  const unsigned long long h = atomicAdd(P.n_relist, 1ull);
  __hip_atomic_store((C2D_GLOBAL int32_t*)(P.relist + h), id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void census_chunk_store(const KParams& P0, int w, uint32_t lane) {
  const KParams& P = cold(P0);
  if (lane != 0) return;
  if (P.clist)
    for (uint32_t i = 0; i < c2d_fs_n[w]; i++) census_relist(P, c2d_fs[w][i]);
  const uint32_t used = c2d_cch_used[w];
  const unsigned long long base = c2d_cch_base[w];
  const int64_t ws = (int64_t)blockIdx.x * (C2D_TR_BLOCK / 64) + w;
  const bool part = used < P.cens_chunk && base < (unsigned long long)P.cap_cout;
  gst(P.cstate + 2 * ws, part ? (int64_t)base : (int64_t)-1);
  gst(P.cstate + 2 * ws + 1, (int64_t)used);
}

/* chunked census, bundle kernel (lane 0): the wave took the work chunk that
 * holds the n census items of (physical) chunk id.  Count-down slots in LDS,
 * open-addressed from id mod C2D_CT_TRACK (a wave has 2-3 chunks in flight:
 * the first probe nearly always hits; r03's direct-mapped table lost ~6 % of
 * the chunks to index collisions).  Only a chunk that finds all
 * slots busy is not counted down and waits for the next step. */
__device__ __forceinline__ void census_track(int w, int32_t id, uint32_t n) {
#pragma unroll 1
  for (int k = 0; k < C2D_CT_TRACK; k++) {
    const int e = (id + k) & (C2D_CT_TRACK - 1);
    if (c2d_ct_idx[w][e] < 0) {
      c2d_ct_idx[w][e] = id;
      c2d_ct_rem[w][e] = n;
      return;
    }
  }
  atomicAdd(&c2d_cnt_lds[C2D_CNT_CLOST_INT], 1u);
}

/* the census source in slot `slot` finished: the last one of its chunk frees
 * the chunk */
C2D_COLD_FN void census_item_done(const KParams& P0, long long slot) {
  const KParams& P = cold(P0);
  const int w = (int)(threadIdx.x >> 6);
  const int32_t id = (int32_t)(slot >> C2D_CCHUNK_LOG);
  int e = id & (C2D_CT_TRACK - 1);
  if (c2d_ct_idx[w][e] != id) {
    /* open addressing: probe on from the home slot */
    int k = 1;
#pragma unroll 1
    for (; k < C2D_CT_TRACK; k++)
      if (c2d_ct_idx[w][(id + k) & (C2D_CT_TRACK - 1)] == id) break;
    if (k == C2D_CT_TRACK) return;                     /* not tracked */
    e = (id + k) & (C2D_CT_TRACK - 1);
  }
  if (atomicSub(&c2d_ct_rem[w][e], 1u) != 1u) return;
  c2d_ct_idx[w][e] = -1;
  const uint32_t s = atomicAdd(&c2d_fs_n[w], 1u);
  if (s < C2D_CT_STACK) {
    c2d_fs[w][s] = id;
  } else {
    atomicSub(&c2d_fs_n[w], 1u);
    census_relist(P, id);
  }
  atomicAdd(&c2d_cnt_lds[C2D_CNT_CREUSE_INT], 1u);
}

/* census write (src/imctrk2d.f:528-578): appended to the wave's chunk */
C2D_COLD_FN void census_write(const KParams& P0, const Tal& T, const Pkt& p, LaneCnt& lc) {
  const KParams& P = cold(P0);
  const Geo* g = T.g;
  int cell = (p.jph - 1) * P.nr + (p.kph - 1);
  cell_add(P, T, TC_NPCEN, cell, 1.0);
  cell_add(P, T, TC_ECENS, cell, p.ew);
#if defined(C2D_ABLATE_NFIELD) && C2D_ABLATE_NFIELD == 1   /* profiling ablations only */
  if (p.xnu < 0.0) {
#else
  int efl = 0;                          /* the record's E_field bin (c2d_cens_jk) */
  if (p.xnu > P.egg_min) {              /* Egg_min = E_field(1)^2/E_field(2), host-computed */
#endif
    const int known = (p.ie >> 16) - 1;
    const int i = known >= 0 ? known : grid_lookup(g->E_field, C2D_NPHFIELD, g->efl_start, g->efl_k0, p.xnu);
    efl = i;
    const double v = FDIV_POS(6.25e8 * p.ew, p.xnu);
#if defined(C2D_ABLATE_NFIELD) && C2D_ABLATE_NFIELD == 2   /* the lookup without the add */
    if (v == 1.25e300)
#endif
#if defined(C2D_ABLATE_NFIELD) && C2D_ABLATE_NFIELD == 3   /* a plain store in place of the add */
    gst(&P.nf_rep[(int64_t)(blockIdx.x % C2D_NF_REPL) * P.ncell * C2D_NPHFIELD +
                  (int64_t)cell * C2D_NPHFIELD + (i - 1)], v);
    if (v == 1.25e300)
#endif
    gadd(&P.nf_rep[(int64_t)(blockIdx.x % C2D_NF_REPL) * P.ncell * C2D_NPHFIELD +
                   (int64_t)cell * C2D_NPHFIELD + (i - 1)], v);
  }
  const unsigned long long slot = census_slot_chunk(P);
  if (slot < (unsigned long long)P.cap_cout) {
    CENS_ST2(P.cout.rz + slot, p.rpre, p.zpre);
#if C2D_TABLE_COMTOT
    CENS_ST2(P.cout.wp + slot, p.wmu, p.eta);        /* encoded azimuth (CensusSoA) */
#else
    CENS_ST2(P.cout.wp + slot, p.wmu, p.phi);
#endif
    CENS_ST2(P.cout.ex + slot, p.ew, p.xnu);
    CENS_ST4(P.cout.tg + slot, c2d_cens_jk(p.jph, p.kph, p.ie & 0xffff, efl),
         (p.bins & 0x00ffffffu)
#if C2D_TABLE_COMTOT
             | (p.esw == -1 ? C2D_CENS_ESW : 0u)
#endif
         , c2d_census_key(p.key, p.ctr, p.sub));
  } else {
    gor(P.err, ERR_CENSUS);
  }
  LC_ADD(lc, C2D_CNT_CENSUS);
}

__device__ __forceinline__ void push_scat(const KParams& P0, ScatRec* q, unsigned long long* n, const ScatRec& r) {
  const KParams& P = cold(P0);
  unsigned long long slot = wave_reserve(n);
  if (slot < (unsigned long long)P.cap_q) {
    q[slot] = r;
  } else {
    gor(P.err, ERR_QUEUE);
  }
}

__device__ __forceinline__ ScatRec make_rec(const Pkt& p, uint64_t key, uint32_t ctr) {
  ScatRec r;
  r.rpre = p.rpre; r.zpre = p.zpre; r.wmu = p.wmu; r.phi = p.phi; r.ew = p.ew; r.xnu = p.xnu;
  r.dcen = p.dcen;
  r.jk = ((uint32_t)p.jph << 16) | (uint32_t)p.kph;
  r.ctr = ctr;
  r.key = key;
  r.kap = (uint32_t)KAP(p);
  r.sub = p.sub;
  return r;
}

__device__ __forceinline__ void load_rec(Pkt& p, const ScatRec& r) {
  p.rpre = r.rpre; p.zpre = r.zpre; p.wmu = r.wmu; p.phi = r.phi; p.ew = r.ew; p.xnu = r.xnu;
  p.dcen = r.dcen;
  p.jph = (int32_t)(r.jk >> 16);
  p.kph = (int32_t)(r.jk & 0xffffu);
  p.bins = (p.bins & 0x00ffffffu) | (r.kap << 24);
}

/* ------------------------------------------------------------------ */
/* per-packet caches                                                   */
/* ------------------------------------------------------------------ */
/* E_ph bin and comtot-table position depend on xnu only: computed when a
 * packet starts (source, probe restart, secondary) instead of every step. */
__device__ __forceinline__ void cache_energy(const KParams& P, const Geo* g, Pkt& p, bool have_ie = false) {
  if (!have_ie) p.ie = grid_lookup(g->E_ph, C2D_N_VOL, g->eph_start, g->eph_k0, p.xnu);
#if C2D_TABLE_COMTOT
#if C2D_LNX_F32
  const double s = ((double)(0.69314718f * __builtin_amdgcn_logf((float)p.xnu)) - C2D_COMTAB_U0) * P.comtab_du_inv;
#else
  const double s = (FLOG(p.xnu) - C2D_COMTAB_U0) * P.comtab_du_inv;
#endif
  if (s >= 1.0 && s < (double)(C2D_COMTAB_N - 3)) {
    p.tg = (int32_t)s;
    p.tt = s - (double)p.tg;
  } else {
    p.tg = 0;
    p.tt = 0.0;
  }
#endif
}

/* azimuth bookkeeping.  Exact build: phi as in the reference (cos(phi) each
 * step, acos after the move).  Fast build: carry Eta = cos(phi) and its
 * quadrant switch between steps (cos(acos(E)) = E to an ulp; drops the
 * reference's 4e-11 rad/step rotation from pi = 3.1415926536), and
 * materialise phi only when an event needs it. */
__device__ __forceinline__ void set_phi(Pkt& p, double phi) {
  p.phi = phi;
#if C2D_TABLE_COMTOT
  p.eta = c2d_cos(phi);
  p.esw = (phi <= PI_REF && phi >= 1.0e-10) ? 1 : -1;
#endif
}

/* ------------------------------------------------------------------ */
/* one packet-step: label 100 ... 900 of src/imctrk2d.f:139-578          */
/* ------------------------------------------------------------------ */
struct ComCache {
  int32_t cell0, cell1;
  double v0, v1;
};

/* -DC2D_TR_PROF: wave-level section timers (shader clock) and event counts,
 * read back with c2d_transport_prof (tools/tr_prof.py).  Sections: */
enum : int {
  TP_REFILL = 0,    /* work fetch (ballot loop)                          */
  TP_START = 1,     /* load_source / load_pk, cache_energy, set_phi       */
  TP_GEOM = 2,      /* flight: colmfp, comtot, geometry                   */
  TP_ABS = 3,       /* flight: absorption, wmustar sampling, deposits     */
  TP_EVENT = 4,     /* flight: acos, census write, escape, collision      */
  TP_POST = 5,      /* push_scat, probe restart from the source record    */
  TP_PTS = 6,       /* bundle: the survivors' absorption points           */
  TP_CWR = 7,       /* bundle: the escape / census write of the step      */
  TP_ITER = 8,      /* loop iterations (waves)                            */
  TP_LANES = 9,     /* sum of lanes in flight over iterations             */
  TP_GOT_W = 10, TP_GOT_L = 11,       /* new items: waves, lanes        */
  TP_CENS_W = 12, TP_CENS_L = 13,     /* census writes                  */
  TP_LEAK_W = 14, TP_LEAK_L = 15,     /* imcleak calls                  */
  TP_COLL_W = 16, TP_COLL_L = 17,     /* collisions                     */
  TP_RST_W = 18, TP_RST_L = 19,       /* probe restarts                 */
  TP_NWAVE = 20
};
struct Prof {
#ifdef C2D_TR_PROF
  uint64_t acc[C2D_TR_PROF_WORDS];
  uint64_t t;
#endif
};
#ifdef C2D_TR_PROF
#define TP_MARK(pf, i) do { const uint64_t _n = clock64(); (pf).acc[i] += _n - (pf).t; (pf).t = _n; } while (0)
#define TP_COUNT(pf, iw, il) do { (pf).acc[iw] += 1; (pf).acc[il] += __popcll(__ballot(1)); } while (0)
#else
#define TP_MARK(pf, i) do { } while (0)
#define TP_COUNT(pf, iw, il) do { } while (0)
#endif

/* V12: the tracker of src_20121113/imctrk2d.f (c2d_config.trk_variant =
 * C2D_TRK_2012_11; include/compton2d.h): the azimuth update with the path's
 * r-plane projection f, colmfp kept across cell boundaries, clamps at 1.
 * V12 = 0 is src/imctrk2d.f bug for bug (hazard H1). */
template <int V12>
__device__ __forceinline__ int flight(const KParams& P, const Tal& T, Pkt& p, ComCache& cc, LaneCnt& lc,
                                      Prof& pf) {
  const double lim8 = V12 ? 1.0 : 9.9999999e-1, lim9 = V12 ? 1.0 : 0.999999999;
  const Geo* g = T.g;
#if C2D_TABLE_COMTOT && C2D_EARLY_LOADS
  /* the step's table reads (comtot interpolation points, n_e, kappa) are
   * issued before the colmfp draw, so their latency overlaps the Philox
   * block and the log instead of following them */
  const int cell_e = (p.jph - 1) * P.nr + (p.kph - 1);
  const double* tb_e = P.comtab + (int64_t)cell_e * C2D_COMTAB_N + (p.tg > 0 ? p.tg - 1 : 0);
  const double ey0 = gld(tb_e), ey1 = gld(tb_e + 1), ey2 = gld(tb_e + 2), ey3 = gld(tb_e + 3);
  const double ene = gld(P.n_e + cell_e);
  const double ekap = gld((KAP(p) ? P.kappa_s : P.kappa_cv) + (int64_t)cell_e * C2D_N_VOL + ((p.ie & 0xffff) - 1));
#endif
  /* mode 0 uses mb_ran = 1e-10 (imctrk2d.f:150) but never reads colmfp (dcol below) */
  double colmfp = 0.0;
  /* src: label 100 every step; 2012-11: only when the track starts (label
   * 110 after a boundary).  The uniform is never 0: no `goto 100` redraw */
  if (p.mode != 0) colmfp = (V12 && p.nflight != 0) ? p.cmfp : -c2d_log(U(p));
  if (p.ew < 1.0e-40) return FL_END;
  if (++p.nflight > MAX_FLIGHTS) {
    LC_ADD(lc, C2D_CNT_ABORTED);
    return FL_END;
  }
  p.wmu = clampd(p.wmu, lim8);
  const int cell = (p.jph - 1) * P.nr + (p.kph - 1);
  double comac = 0.0;
  if (p.mode != 0) {
#if C2D_TABLE_COMTOT && C2D_EARLY_LOADS
    comac = (p.tg == 0) ? comtot_exact(P, cell, p.xnu)
                        : comtot_interp(ey0, ey1, ey2, ey3, ene, p.tt);
    (void)cc;
#elif C2D_TABLE_COMTOT
    comac = comtot_table(P, cell, p.xnu, p.tg, p.tt);
    (void)cc;
#else
    /* comtot is a pure function of (cell, xnu): caching per packet is exact
     * (the reference caches per imctrk2d(-1) call, imctrk2d.f:170-178) */
    if (cc.cell0 == cell) {
      comac = cc.v0;
    } else if (cc.cell1 == cell) {
      comac = cc.v1;
    } else {
      comac = comtot_exact(P, cell, p.xnu);
      cc.cell1 = cc.cell0; cc.v1 = cc.v0;
      cc.cell0 = cell; cc.v0 = comac;
    }
#endif
  }
  const double sigsc = comac;
  const double rkm1 = (p.kph == 1) ? P.rmin : g->r[p.kph - 1];
  const double xqsqleft = rkm1 * rkm1;
  double dcol;
  if (p.mode != 0)
    dcol = colmfp / sigsc;
  else
    dcol = 100 * (g->r[P.nr] > g->z[P.nz] ? g->r[P.nr] : g->z[P.nz]);
  double trld;
  int ikind;
  if (p.dcen <= dcol) { trld = p.dcen; ikind = 2; }
  else { trld = dcol; ikind = 3; }
  lc.steps++;
  /* geometry (imctrk2d.f:228-379) */
#if C2D_TABLE_COMTOT
  double Eta = p.eta;
  const int eta_switch = p.esw;
#else
  double Eta = c2d_cos(p.phi);
  const int eta_switch = (p.phi <= PI_REF && p.phi >= 1.0e-10) ? 1 : -1;
#endif
  if (!V12) Eta = clampd(Eta, lim8);          /* commented out in src_20121113:248-249 */
  const double rpre = p.rpre, zpre = p.zpre, wmu = p.wmu;
  const double disp = Eta * rpre;
  const double psq = rpre * rpre * (1.0 - Eta * Eta);
  int kbnd, inout, knew, jnew;
  double rbnd, Zbnd;
  if (Eta < 0.0 && psq < xqsqleft) {
    kbnd = p.kph - 1;
    inout = -1;
    rbnd = rkm1;
  } else {
    kbnd = p.kph;
    inout = 1;
    rbnd = g->r[p.kph];
  }
  double dpbsq = rbnd * rbnd - psq;
  if (dpbsq < 1.0e-6) dpbsq = 1.0e-6;
  const double disbr = (double)inout * __builtin_sqrt(dpbsq) - disp;
  const double swmu = __builtin_sqrt(1.0 - wmu * wmu);
  double trldb = disbr / swmu;
  double fr = disbr;                           /* the reference's f (imctrk2d.f:278,290,380) */
  const double Zr = zpre + wmu * trldb;
  const double zlow = (p.jph == 1) ? P.zmin : g->z[p.jph - 1];
  const double zup = g->z[p.jph];
  if (Zr > zup || Zr < zlow) {
    Zbnd = (Zr > zup) ? zup : zlow;
    knew = p.kph;
    jnew = (Zr > zup) ? p.jph + 1 : p.jph - 1;
    const double f = (Zbnd - zpre) * swmu / wmu;
    fr = f;
    rbnd = __builtin_sqrt(rpre * rpre + f * f + 2.0 * rpre * f * Eta);
    trldb = __builtin_sqrt(f * f + (Zbnd - zpre) * (Zbnd - zpre));
  } else {
    knew = p.kph + inout;
    jnew = p.jph;
    rbnd = (kbnd > 0) ? g->r[kbnd] : P.rmin;
    Zbnd = Zr;
  }
  double rnew, znew;
  if (trldb < trld) {
    ikind = 1;
    trld = trldb;
    rnew = rbnd;
    znew = Zbnd;
  } else {
    jnew = p.jph;
    knew = p.kph;
    const double f = trld * swmu;
    fr = f;
    rnew = __builtin_sqrt(f * f + rpre * rpre + 2.0 * f * rpre * Eta);
    znew = zpre + trld * wmu;
  }
  TP_MARK(pf, TP_GEOM);
  /* absorption (imctrk2d.f:382-462); gamma-gamma opacity inert (H6) */
#if C2D_TABLE_COMTOT && C2D_EARLY_LOADS
  double sigabs = 1.0e-40 + 1.0 * ekap;
#else
  const double* kap = KAP(p) ? P.kappa_s : P.kappa_cv;
  double sigabs = 1.0e-40 + 1.0 * gld(kap + (int64_t)cell * C2D_N_VOL + ((p.ie & 0xffff) - 1));
#endif
  if (sigabs < 1.0e-40) sigabs = 1.0e-40;
  const double xabs = sigabs * trld;
  const double ewnew = (xabs < 100.0) ? p.ew * c2d_exp(-xabs) : 0.0;
  double deleabs = p.ew - ewnew;
  if (deleabs < 1.0e-50) deleabs = 1.0e-50;
  double wmustar;
  if (xabs <= 0.00001) {
    wmustar = wmu;
  } else {
    double mr, sstar = 0.0;
    for (int guard = 0; guard < MAX_REJECT; guard++) {
      mr = U(p);
      if (mr < p.ew / deleabs) {
        sstar = -c2d_log(1.0 - mr * deleabs / p.ew) / sigabs;
        break;
      }
    }
    const double denom = __builtin_sqrt(rpre * rpre + 2.0 * wmu * rpre * sstar + sstar * sstar);
    wmustar = (wmu * rpre + sstar) / denom;
  }
  const double delpr = deleabs * wmustar * C_LIGHT;
  if (p.mode != 0) {
    cell_add(P, T, TC_EDEP, cell, deleabs);
    cell_add(P, T, TC_PRDEP, cell, delpr);
  }
  TP_MARK(pf, TP_ABS);
  if (ewnew <= p.wtmin) {
    LC_ADD(lc, C2D_CNT_KILLED);
    return FL_END;
  }
  p.ew = ewnew;
  p.dcen = p.dcen - trld;
  if (V12)
    Eta = (fr + Eta * rpre) / rnew;          /* src_20121113/imctrk2d.f:478 */
  else
    Eta = (trld + Eta * rpre) / rnew;        /* hazard H1: trld, not f (imctrk2d.f:472) */
  Eta = clampd(Eta, lim9);
  if (V12 && ikind == 1) p.cmfp = colmfp - sigsc * trld;   /* src_20121113/imctrk2d.f:505 */
  const bool leaves = (jnew == P.nz + 1 || jnew == 0 || knew == P.nr + 1 || knew == 0);
#if C2D_TABLE_COMTOT
  p.eta = Eta;
  if (p.mode != -1 && (ikind == 3 || leaves)) {   /* an event will read phi (census: encoded) */
    p.phi = c2d_acos(Eta);
    if (eta_switch == -1) p.phi = 2.0 * PI_REF - p.phi;
  }
#else
  p.phi = c2d_acos(Eta);
  if (eta_switch == -1) p.phi = 2.0 * PI_REF - p.phi;
#endif
  p.rpre = rnew;
  p.zpre = znew;
  if (ikind == 1) {
    if (leaves) {
      p.jph = jnew;
      p.kph = knew;
      if (p.mode == -1) return FL_END;
      TP_COUNT(pf, TP_LEAK_W, TP_LEAK_L);
      if (imcleak(P, T, p, lc) == 1) {
        if (p.mode == 1) LC_ADD(lc, C2D_CNT_ESC_SCAT);
        return FL_END;
      }
      set_phi(p, p.phi);                        /* axis pass-through set phi = 1e-6 */
      return FL_CONT;
    }
    p.kph = knew;
    p.jph = jnew;
    return FL_CONT;
  }
  if (ikind == 2) {
    if (p.mode != -1) {
      TP_COUNT(pf, TP_CENS_W, TP_CENS_L);
      census_write(P, T, p, lc);
    }
    return FL_END;
  }
  LC_ADD(lc, C2D_CNT_COLLIDE);
  TP_COUNT(pf, TP_COLL_W, TP_COLL_L);
  if (p.mode == -1) {   /* probes read phi too (the collision record) */
#if C2D_TABLE_COMTOT
    p.phi = c2d_acos(Eta);
    if (eta_switch == -1) p.phi = 2.0 * PI_REF - p.phi;
#endif
  }
  return FL_COLLIDE;
}

/* ------------------------------------------------------------------ */
/* sources                                                             */
/* ------------------------------------------------------------------ */
/* A source being sampled: sub-stream 0 from counter 0, so draw n is output n
 * of the SplitMix64 sequence seeded with the key (c2d_stream64); `zs` carries
 * that sequence's state, key + (n + 1)*gamma, and a draw adds gamma instead
 * of multiplying it by the counter (the same outputs as U(Pkt&)). */
struct SrcPkt : Pkt {
  uint64_t zs;
};
__device__ __forceinline__ void src_seed(SrcPkt& p) { p.zs = p.key + 0x9E3779B97F4A7C15ull; }
__device__ __forceinline__ double U(SrcPkt& p) {
  const uint64_t x = c2d_mix64(p.zs);
  p.zs += 0x9E3779B97F4A7C15ull;
  return c2d_u01_bits((uint32_t)(x >> 32), (uint32_t)x);
}

/* planck (src/planck2d.f:1-141) */
__device__ __forceinline__ void planck(const KParams& P, const Geo* G, SrcPkt& p, double tpl) {
  double u4, ap0, ap1 = 1.0, ap2 = 1.0, ap3 = 1.0, rn1;
  do {
    u4 = U(p);
    u4 = u4 * U(p);
    u4 = u4 * U(p);
    u4 = u4 * U(p);
  } while (u4 <= 1.0e-200);
  ap0 = -c2d_log(u4);
  rn1 = 1.08232 * U(p);
  while (!(rn1 <= ap1)) {
    ap2 = ap2 + 1.0;
    ap3 = 1.0 / ap2;
    ap1 = ap1 + (ap3 * ap3) * (ap3 * ap3);
  }
  p.xnu = ap0 * ap3 * tpl;
  set_bins(p, bin_sp(G, P.nphtotal, p.xnu, F32(1.000001), F32(0.999999), 0), bin_lc(G, P.nph_lc, p.xnu),
           bin_mu(G, P.nmu, p.wmu));
}

/* file_sample (src/imcsurf2d_para.f:694-788) */
__device__ __forceinline__ void file_sample(const KParams& P, const Geo* G, SrcPkt& p, int spec) {
  if (spec < 0 || spec >= P.n_spectra) {
    gor(P.err, ERR_SPEC);
    p.xnu = 1.0;
    set_bins(p, 0, 0, bin_mu(G, P.nmu, p.wmu));
    return;
  }
  const SpecDev sp = P.spectra[spec];
  double x1 = U(p);
  int i;
  for (i = 1; i <= sp.nfile - 1; i++)
    if (sp.P_file[i - 1] > x1) break;
  if (i > sp.nfile - 1) i = sp.nfile - 1;
  double x2 = U(p);
  double Ei = sp.E_file[i - 1], a1 = sp.a1[i - 1], Ii = sp.I_file[i - 1], Fi = sp.F_file[i - 1];
  p.xnu = Ei * c2d_pow(a1 * Ii * x2 / (Fi * Ei) + 1.0, 1.0 / a1);
  set_bins(p, bin_sp(G, P.nphtotal, p.xnu, 1.000001, 0.999999, 0), bin_lc(G, P.nph_lc, p.xnu),
           bin_mu(G, P.nmu, p.wmu));
}

/* one volume packet of vol_calc (src/imcvol2d_para.f:157-392) */
__device__ __forceinline__ void vol_source(const KParams& P, const Geo* g, SrcPkt& p, int jv, int kv) {
  const int cell = (jv - 1) * P.nr + (kv - 1);
  const double* vf = P.vfrac + 4 * cell;
  const double f_thermal = vf[0], f_inn = vf[1], f_outer = vf[2], f_upper = vf[3];
  const double rlow = (kv == 1) ? P.rmin : g->r[kv - 1];
  p.jph = jv;
  p.kph = kv;
  p.ew = P.ewsv[cell];
  p.dcen = C_LIGHT * P.dt * U(p);
  double rnum = U(p), psi;
  if (rnum < f_thermal) {
    rnum = U(p);
    int i = cdf_index(P.eps_th + (int64_t)cell * C2D_N_VOL, C2D_N_VOL, rnum, P.eps_linear,
                      P.cdf_guide ? P.cdf_guide + (int64_t)(P.ncell + cell) * (C2D_CDF_GUIDE + 1) : nullptr);
    if (i < C2D_N_VOL) p.xnu = g->E_ph[i] + U(p) * (g->E_ph[i + 1] - g->E_ph[i]);
    else p.xnu = g->E_ph[i];
    double rnum0 = U(p);
    if (rnum0 < f_inn) {
      p.wmu = clampd(2.0 * U(p) - 1.0, 9.9999999e-1);
      double x1 = U(p), x2 = U(p);
      if (x1 < 0.5) {
        p.phi = 1.1e1 / 7.0 + (1.1e1 / 7.0) * x2;
        if (p.phi < 1.57079638) p.phi = 1.57079638;
      } else {
        p.phi = -1.1e1 / 7.0 - (1.1e1 / 7.0) * x2;
        if (p.phi > -1.57079638) p.phi = -1.57079638;
      }
      p.rpre = (kv == 1) ? F32(1.00001) * P.rmin : F32(1.00001) * g->r[kv - 1];
      p.zpre = (jv == 1) ? g->z[1] * U(p) : g->z[jv - 1] + U(p) * (g->z[jv] - g->z[jv - 1]);
    } else if (rnum0 < f_outer) {
      p.wmu = clampd(2.0 * U(p) - 1.0, 9.9999999e-1);
      p.rpre = F32(0.999999) * g->r[kv];
      p.zpre = (jv == 1) ? g->z[1] * U(p) : g->z[jv - 1] + U(p) * (g->z[jv] - g->z[jv - 1]);
      p.phi = -1.1e1 / 7.0 + 2.2e1 / 7.0 * U(p);
      if (p.phi < -1.5707963) p.phi = -1.57079063;
      if (p.phi > 1.5707963) p.phi = 1.5707963;
    } else if (rnum0 < f_upper) {
      p.wmu = U(p);
      if (p.wmu > 9.9999999e-1) p.wmu = 9.9999999e-1;
      if (p.wmu < 0.0) p.wmu = 0.0;
      p.phi = 4.4e1 / 7.0 * U(p);
      if (p.phi > 2.0 * PI_REF) p.phi = 2.0 * PI_REF;
      psi = U(p);
      p.zpre = F32(0.999999) * g->z[jv];
      p.rpre = __builtin_sqrt(rlow * rlow + psi * (g->r[kv] * g->r[kv] - rlow * rlow));
    } else {
      p.wmu = -U(p);
      p.phi = 4.4e1 / 7.0 * U(p);
      if (p.wmu > 0.0) p.wmu = 0.0;
      if (p.wmu < -9.9999999e-1) p.wmu = -9.9999999e-1;
      if (p.phi > 2.0 * PI_REF) p.phi = 2.0 * PI_REF;
      if (jv == 1) {
        p.zpre = F32(1.000001) * P.zmin;
        if (p.zpre <= P.zmin) p.zpre = P.zmin + 1.0e-6;
      } else {
        p.zpre = F32(1.000001) * g->z[jv - 1];
        if (p.zpre <= g->z[jv - 1]) p.zpre = g->z[jv - 1] + 1.0e-6;
      }
      psi = U(p);
      p.rpre = __builtin_sqrt(rlow * rlow + psi * (g->r[kv] * g->r[kv] - rlow * rlow));
    }
  } else {
    rnum = U(p);
    int i = cdf_index(P.eps_tot + (int64_t)cell * C2D_N_VOL, C2D_N_VOL, rnum, P.eps_linear,
                      P.cdf_guide ? P.cdf_guide + (int64_t)cell * (C2D_CDF_GUIDE + 1) : nullptr);
    if (i < C2D_N_VOL) p.xnu = g->E_ph[i] + U(p) * (g->E_ph[i + 1] - g->E_ph[i]);
    else p.xnu = g->E_ph[i];
    p.wmu = 2.0 * U(p) - 1.0;
    p.phi = 4.4e1 / 7.0 * U(p);
    p.wmu = clampd(p.wmu, 9.9999999e-1);
    if (p.phi > 2.0 * PI_REF) p.phi = 2.0 * PI_REF;
    p.zpre = (jv == 1) ? g->z[1] * U(p) : g->z[jv - 1] + U(p) * (g->z[jv] - g->z[jv - 1]);
    psi = U(p);
    p.rpre = __builtin_sqrt(rlow * rlow + psi * (g->r[kv] * g->r[kv] - rlow * rlow));
  }
  set_bins(p, bin_sp(g, P.nphtotal, p.xnu, F32(1.000001), F32(0.999999), P.nphtotal),
           bin_lc(g, P.nph_lc, p.xnu), bin_mu(g, P.nmu, p.wmu));
}

/* surface packets: z_surf_calc / r_surf_calc (src/imcsurf2d_para.f:254-528).
 * side 0 inner z-surface js, 1 outer js, 2 upper r-surface ks, 3 lower ks. */
__device__ __forceinline__ void surf_source(const KParams& P, const Geo* g, SrcPkt& p, int side, int s1, int slot) {
  const double lim10 = 0.9999999999;
  const double ew = P.surf_ew[slot], tbb = P.surf_tbb[slot];
  const int spec = P.surf_spec[slot];
  if (side == 0) {
    const int js = s1;
    p.jph = js;
    p.wmu = clampd(2.0 * U(p) - 1.0, lim10);
    p.phi = -1.1e1 / 7.0 + 2.2e1 / 7.0 * U(p);
    if (p.phi < -1.5707963) p.phi = -1.57079063;
    if (p.phi > 1.5707963) p.phi = 1.5707963;
    p.rpre = P.rmin;
    p.zpre = (js == 1) ? g->z[1] * U(p) : g->z[js - 1] + U(p) * (g->z[js] - g->z[js - 1]);
    p.ew = ew;
    p.dcen = U(p) * C_LIGHT * P.dt;
    if (tbb > 0.0) planck(P, g, p, tbb);
    else file_sample(P, g, p, spec);
    p.kph = 1;
  } else if (side == 1) {
    const int js = s1;
    p.jph = js;
    p.wmu = clampd(2.0 * U(p) - 1.0, lim10);
    p.rpre = g->r[P.nr];
    p.zpre = (js == 1) ? g->z[1] * U(p) : g->z[js - 1] + U(p) * (g->z[js] - g->z[js - 1]);
    double x1 = U(p), x2 = U(p);
    if (x1 < 0.5) {
      p.phi = 1.1e1 / 7.0 + (1.1e1 / 7.0) * x2;
      if (p.phi < 1.57079638) p.phi = 1.57079638;
    } else {
      p.phi = -1.1e1 / 7.0 - (1.1e1 / 7.0) * x2;
      if (p.phi > -1.57079638) p.phi = -1.57079638;
    }
    p.ew = ew;
    p.dcen = U(p) * C_LIGHT * P.dt;
    if (tbb > 0.0) planck(P, g, p, tbb);
    else file_sample(P, g, p, spec);
    p.kph = P.nr;
  } else {
    const int ks = s1;
    const double rlow = (ks == 1) ? P.rmin : g->r[ks - 1];
    p.kph = ks;
    if (side == 2) {
      p.wmu = clampd(-U(p), lim10);
      p.phi = 2.0 * PI_REF * U(p);
      double psi = U(p);
      p.zpre = g->z[P.nz];
      p.rpre = __builtin_sqrt(rlow * rlow + psi * (g->r[ks] * g->r[ks] - rlow * rlow));
      p.ew = ew;
      p.dcen = U(p) * C_LIGHT * P.dt;
      if (tbb > 0.0) planck(P, g, p, tbb);
      else file_sample(P, g, p, spec);
      p.jph = P.nz;
    } else {
      p.wmu = 9.9999999e-1;
      p.phi = 2.0 * PI_REF * U(p);
      double psi = U(p);
      p.zpre = P.zmin;
      p.rpre = __builtin_sqrt(rlow * rlow + psi * (g->r[ks] * g->r[ks] - rlow * rlow));
      p.ew = ew;
      if (tbb > 0.0) planck(P, g, p, tbb);
      else file_sample(P, g, p, spec);
      p.dcen = U(p) * C_LIGHT * P.dt;
      p.jph = 1;
    }
  }
}

__device__ __forceinline__ int upper_index(const int64_t* prefix, int n, int64_t gidx) {
  /* largest c in [0, n) with prefix[c] <= gidx */
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= gidx) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ void init_counters(uint32_t* sh) {
  if (threadIdx.x < C2D_NCOUNTERS) sh[threadIdx.x] = 0u;
}

/* after the final __syncthreads of the kernel */
__device__ __forceinline__ void flush_counters(const KParams& P, LaneCnt& lc, uint32_t lane) {
  const uint32_t st = wave_sum(lc.steps);
  const uint32_t pa = wave_sum(lc.paths);
  if (lane == 0 && st) atomicAdd(&c2d_cnt_lds[C2D_CNT_STEPS], st);
  if (lane == 0 && pa) atomicAdd(&c2d_cnt_lds[C2D_CNT_PATHS_INT], pa);
  __syncthreads();
  if (threadIdx.x < C2D_NCOUNTERS && c2d_cnt_lds[threadIdx.x])
    atomicAdd(&P.cnt[threadIdx.x], (unsigned long long)c2d_cnt_lds[threadIdx.x]);
}

__device__ __forceinline__ void store_pk(const PktSoA& s, int64_t i, const Pkt& p) {
  s.rpre[i] = p.rpre; s.zpre[i] = p.zpre; s.wmu[i] = p.wmu; s.phi[i] = p.phi;
  s.ew[i] = p.ew; s.xnu[i] = p.xnu; s.dcen[i] = p.dcen;
  s.jk[i] = ((uint32_t)p.jph << 16) | (uint32_t)p.kph;
  s.bins[i] = p.bins;
  s.ctr[i] = p.ctr;
  s.sub[i] = p.sub;
  s.key[i] = p.key;
}

__device__ __forceinline__ void load_pk(Pkt& p, const PktSoA& s, int64_t i) {
  p.rpre = gld(s.rpre + i); p.zpre = gld(s.zpre + i); p.wmu = gld(s.wmu + i); p.phi = gld(s.phi + i);
  p.ew = gld(s.ew + i); p.xnu = gld(s.xnu + i); p.dcen = gld(s.dcen + i);
  const uint32_t jk = gld(s.jk + i), bn = gld(s.bins + i);
  p.jph = (int32_t)(jk >> 16); p.kph = (int32_t)(jk & 0xffffu);
  p.bins = bn;
  p.ctr = gld(s.ctr + i);
  p.key = gld(s.key + i);
  p.sub = gld(s.sub + i);
}

}  // namespace

/* ------------------------------------------------------------------ */
/* generation-0 sources: volume (imcvol2d_para.f:90-414) and surface     */
/* (imcsurf2d_para.f:228-534) packets, one lane per packet               */
/* ------------------------------------------------------------------ */
__global__ void __launch_bounds__(SRCBLOCK) C2D_SFX(c2d_source_kernel)(const KParams* __restrict__ Pg) {
  const KParams& P = *Pg;
  __shared__ double geo_lds[GEO_DOUBLES];
  /* the volume-source prefix over cells, for the per-packet cell search
   * (9-10 dependent probes): in LDS when it fits */
  constexpr int PREF_LDS = 1100;
  __shared__ int64_t pref_lds[PREF_LDS];
  const bool pref_in_lds = P.ncell + 1 <= PREF_LDS;
  {
    const double* gsrc = reinterpret_cast<const double*>(P.geo);
    for (int i = threadIdx.x; i < GEO_DOUBLES; i += SRCBLOCK) geo_lds[i] = gsrc[i];
    if (pref_in_lds)
      for (int i = threadIdx.x; i <= P.ncell; i += SRCBLOCK) pref_lds[i] = P.vol_prefix[i];
  }
  __syncthreads();
  const Geo* g = reinterpret_cast<const Geo*>(geo_lds);
  const int64_t n = P.n_vol_items + P.n_surf_items;
  const int64_t stride = (int64_t)gridDim.x * SRCBLOCK;
  for (int64_t it = (int64_t)blockIdx.x * SRCBLOCK + threadIdx.x; it < n; it += stride) {
    SrcPkt p;
    p.ctr = 0;
    p.sub = 0;
    if (it < P.n_vol_items) {
      const int64_t gidx = it * P.world + P.rank;
      int cell;
      int64_t nn;
      if (pref_in_lds) {
        /* upper_index on the LDS copy, once per wave for its first active
         * lane (the smallest gidx: gidx rises with the lane): the other lanes
         * share that cell unless the wave straddles a cell boundary (a cell
         * holds ~1e5 or more sources), and then search for themselves */
        const int64_t gf = (int64_t)rfl64((uint64_t)gidx);
        int lo = 0, hi = P.ncell - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if ((int64_t)rfl64((uint64_t)pref_lds[mid]) <= gf) lo = mid;
          else hi = mid - 1;
        }
        cell = lo;
        if (__ballot(!(gidx < pref_lds[lo + 1])) == 0ull) {
          /* the whole wave in the cell: a wave-uniform cell, so its
           * constants (volume fractions, weight, bounds, CDF rows) are
           * scalar loads */
          const int cu = lo;
          p.key = c2d_derive(P.step_key, C2D_TAG_VOL, (uint32_t)(gidx - pref_lds[cu]), (uint32_t)cu);
          p.bins = 0u;                   /* kap 0: census/volume phase */
          src_seed(p);
          vol_source(P, g, p, cu / P.nr + 1, cu % P.nr + 1);
          goto vol_done;
        }
        if (!(gidx < pref_lds[lo + 1])) {
          lo = 0; hi = P.ncell - 1;
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (pref_lds[mid] <= gidx) lo = mid;
            else hi = mid - 1;
          }
          cell = lo;
        }
        nn = gidx - pref_lds[cell];
      } else {
        cell = upper_index(P.vol_prefix, P.ncell, gidx);
        nn = gidx - P.vol_prefix[cell];
      }
      p.key = c2d_derive(P.step_key, C2D_TAG_VOL, (uint32_t)nn, (uint32_t)cell);
      p.bins = 0u;                       /* kap 0: census/volume phase */
      src_seed(p);
      vol_source(P, g, p, cell / P.nr + 1, cell % P.nr + 1);
    vol_done:;
    } else {
      const int64_t gidx = (it - P.n_vol_items) * P.world + P.rank;
      const int slot = upper_index(P.surf_prefix, P.nslot, gidx);
      const int64_t nn = gidx - P.surf_prefix[slot];
      int side, s1;
      if (slot < 2 * P.nz) { side = slot & 1; s1 = slot / 2 + 1; }
      else { side = 2 + ((slot - 2 * P.nz) & 1); s1 = (slot - 2 * P.nz) / 2 + 1; }
      p.key = c2d_derive(P.step_key, C2D_TAG_SURF + (uint32_t)side, (uint32_t)nn,
                         (uint32_t)(s1 - 1));
      p.bins = 1u << 24;                 /* kap 1: surface phase */
      src_seed(p);
      surf_source(P, g, p, side, s1, slot);
    }
    p.ctr = 0;   /* a source's own draws are done: its copies use sub-streams */
    if (P.vol_cens_base >= 0) {
      if (it < P.n_vol_items) {
        /* census format (pf_apply reads it back; C2D_CENS_VOL: dcen from the key) */
        const int64_t s = P.vol_cens_base + it;
        CENS_ST2(P.cin.rz + s, p.rpre, p.zpre);
#if C2D_TABLE_COMTOT
        const double eta = c2d_cos(p.phi);           /* set_phi's encoding (CensusSoA) */
        const bool esw_neg = !(p.phi <= PI_REF && p.phi >= 1.0e-10);
        CENS_ST2(P.cin.wp + s, p.wmu, eta);
#else
        const bool esw_neg = false;
        CENS_ST2(P.cin.wp + s, p.wmu, p.phi);
#endif
        CENS_ST2(P.cin.ex + s, p.ew, p.xnu);
        const int ie = grid_lookup(g->E_ph, C2D_N_VOL, g->eph_start, g->eph_k0, p.xnu);
        const int efl = p.xnu > P.egg_min ? grid_lookup(g->E_field, C2D_NPHFIELD, g->efl_start, g->efl_k0, p.xnu) : 0;
        CENS_ST4(P.cin.tg + s, c2d_cens_jk(p.jph, p.kph, ie, efl),
                 (p.bins & 0x00ffffffu) | C2D_CENS_VOL | (esw_neg ? C2D_CENS_ESW : 0u), p.key);
      } else {
        store_pk(P.pk, it - P.n_vol_items, p);
      }
    } else {
      store_pk(P.pk, it, p);
    }
  }
}

/* ------------------------------------------------------------------ */
/* scatter secondaries (imctrk2d.f:580-684): one lane per split copy     */
/* ------------------------------------------------------------------ */
/* A split3 copy resamples its scatter until the gain exceeds the trigger
 * (imctrk2d.f:634-648, `goto 215`): attempt k draws from sub-stream k of the
 * copy's key (c2d_rng.h), so attempts are independent.  The scatter kernel
 * runs a copy's first GenArgs.sc_k1 (16) attempts on its own lane; a copy still below the
 * trigger (a gain the electron tail reaches with probability ~1e-3..1e-6)
 * goes to the hard list, whose copies c2d_scatter_hard_kernel resamples 64
 * attempts at a time, one wave per copy: a single long chain no longer holds
 * a whole launch (Compton workload: 98.9 % of the GPU time was one lane's
 * chain in the scatter kernel, profiles/r09i). */

struct ScatItem {
  ScatRec rec;
  uint32_t ii;
  bool is2;
};
__device__ __forceinline__ ScatItem scat_item(const KParams& P, const GenArgs& A, int64_t item) {
  const int64_t n2items = A.n2_in * P.split2;
  ScatItem s;
  s.is2 = item < n2items;
  if (s.is2) {
    s.rec = A.q2_in[item / P.split2];
    s.ii = (uint32_t)(item % P.split2);
  } else {
    const int64_t it3 = item - n2items;
    s.rec = A.q3_in[it3 / P.split3];
    s.ii = (uint32_t)(it3 % P.split3);
  }
  return s;
}

/* one attempt (wave-uniform call): the copy's state at the collision,
 * weight ewold, sub-stream k; lanes with run = false only cooperate */
template <int TALLY = 1>
__device__ __forceinline__ int scat_attempt(const KParams& P, const Geo* g, double* nel, Pkt& p,
                                            const ScatRec& rec, uint64_t key, uint32_t k, double ewold,
                                            bool run, int kn_cap) {
  if (run) {
    p.key = key;
    p.sub = k;
    p.ctr = 0;
    load_rec(p, rec);
    p.ew = ewold;
  }
  return compb2d_w<TALLY>(P, g, nel, p, run, kn_cap);
}

/* the scattered copy: edep / E_IC, then into the packet store for this
 * generation's transport launch (imctrk2d.f:649-660, 664-678) */
__device__ __forceinline__ void scat_emit(const KParams& P, const GenArgs& A, double* eic, Pkt& p, int i_gam,
                                          double ewold) {
  const double twopi = 2.0 * PI_REF;
  const int cell = (p.jph - 1) * P.nr + (p.kph - 1);
  atomicAdd(&P.T[P.off.edep + cell], p.ew - ewold);
  atomicAdd(&eic[i_gam], p.ew - ewold);
  if (p.phi > twopi) p.phi = p.phi - twopi;
  const unsigned long long slot = wave_reserve(A.n_pk);
  if (slot < (unsigned long long)P.cap_pk) store_pk(P.pk, (int64_t)slot, p);
  else gor(P.err, ERR_QUEUE);
}

__global__ void __launch_bounds__(SBLOCK) C2D_SFX(c2d_scatter_kernel)(const KParams* __restrict__ Pg,
                                                                     const GenArgs A) {
  const KParams& P = *Pg;
  __shared__ double geo_lds[GEO_DOUBLES];
  __shared__ double nel_lds[C2D_NUM_NT + 2];
  __shared__ double eic_lds[C2D_NUM_NT + 2];
  for (int i = threadIdx.x; i < GEO_DOUBLES; i += SBLOCK)
    geo_lds[i] = reinterpret_cast<const double*>(P.geo)[i];
  for (int i = threadIdx.x; i < C2D_NUM_NT + 2; i += SBLOCK) {
    nel_lds[i] = 0.0;
    eic_lds[i] = 0.0;
  }
  init_counters(c2d_cnt_lds);
  __syncthreads();
  const Geo* g = reinterpret_cast<const Geo*>(geo_lds);
  LaneCnt lc = {0u};
  const int64_t stride = (int64_t)gridDim.x * SBLOCK;
  const uint32_t lane = lane_id();
  /* split2 copies: one attempt; split3 copies: A.sc_k1 here (0: all to the hard list) */
  const uint32_t sc_k1 = (uint32_t)A.sc_k1;
  const uint32_t k_loop = sc_k1 > 1u ? sc_k1 : 1u;
  /* wave-uniform trip count: compb2d_w cooperates across the wave */
  for (int64_t base = A.item_begin + (int64_t)blockIdx.x * SBLOCK +
                      (int64_t)(__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u);
       base < A.item_end; base += stride) {
    const int64_t item = base + lane;
    const bool act = item < A.item_end;
    ScatItem it;
    it.is2 = true; it.ii = 0;
    double ewold = 0.0, thr = 0.0;
    uint64_t key = 0;
    if (act) {
      it = scat_item(P, A, item);
      const double ewcsv = it.rec.ew / P.split2;
      /* split2 copy: ew = ewcsv; split3 copy: ew = ewcsv / split3 (imctrk2d.f:611,636) */
      ewold = it.is2 ? ewcsv : ewcsv / P.split3;
      thr = ewold * P.split2 * P.split1 * P.spl3_trg;
      key = c2d_derive_s(it.rec.key, it.is2 ? C2D_TAG_SCAT2 : C2D_TAG_SCAT3, it.ii, it.rec.ctr, it.rec.sub);
    }
    /* a split2 copy: one scatter; a split3 copy: resamples until the gain
     * exceeds the trigger, its first sc_k1 attempts here */
    Pkt p;
    int i_gam = 0;
    bool pending = act && (it.is2 || sc_k1 > 0u), done = false;
    for (uint32_t k = 0; k < k_loop; k++) {
      if (__ballot(pending) == 0ull) break;
      if (pending) {
        p.key = key;
        p.sub = k;
        p.ctr = 0;
        load_rec(p, it.rec);
        p.ew = ewold;
      }
      const int ig = compb2d_w(P, g, nel_lds, p, pending, A.kn_cap);
      if (pending) {
        i_gam = ig;
        if (it.is2 || p.ew > thr) { done = true; pending = false; }
        else if (k + 1u >= sc_k1) pending = false;
      }
    }
    if (!act) continue;
    if (it.is2 && p.ew > thr) {   /* third split (imctrk2d.f:631-661): resampled next generation */
      ScatRec r3 = it.rec;
      r3.key = p.key;
      r3.ctr = p.ctr;
      r3.sub = 0;
      push_scat(P, A.q3_out, A.n3_out, r3);
    } else if (done) {
      scat_emit(P, A, eic_lds, p, i_gam, ewold);
    } else {
      const unsigned long long h = wave_reserve(A.n_hard);
      if (h < (unsigned long long)P.cap_pk) A.hard[h] = item;
      else gor(P.err, ERR_QUEUE);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C2D_NUM_NT + 2; i += SBLOCK) {
    if (nel_lds[i] != 0.0) atomicAdd(&P.T[P.off.nelectron + i], nel_lds[i]);
    if (eic_lds[i] != 0.0) atomicAdd(&P.T[P.off.E_IC + i], eic_lds[i]);
  }
  flush_counters(P, lc, lane_id());
}

/* The hard list: one wave per split3 copy, attempts sc_k1 + 64 r + lane in
 * round r.  Every lane's attempt is tallied (nelectron, compb2d calls) as
 * it runs; the first success (lowest lane) is the copy's result, and the
 * lanes after it in that round subtract their attempt's tallies again, so
 * the sums are those of the sequential loop.  Attempt MAX_REJECT ends the
 * copy as the sequential guard does (C2D_CNT_ABORTED). */
__global__ void __launch_bounds__(SBLOCK) C2D_SFX(c2d_scatter_hard_kernel)(const KParams* __restrict__ Pg,
                                                                          const GenArgs A) {
  const KParams& P = *Pg;
  __shared__ double geo_lds[GEO_DOUBLES];
  __shared__ double nel_lds[C2D_NUM_NT + 2];
  __shared__ double eic_lds[C2D_NUM_NT + 2];
  for (int i = threadIdx.x; i < GEO_DOUBLES; i += SBLOCK)
    geo_lds[i] = reinterpret_cast<const double*>(P.geo)[i];
  for (int i = threadIdx.x; i < C2D_NUM_NT + 2; i += SBLOCK) {
    nel_lds[i] = 0.0;
    eic_lds[i] = 0.0;
  }
  init_counters(c2d_cnt_lds);
  __syncthreads();
  const Geo* g = reinterpret_cast<const Geo*>(geo_lds);
  LaneCnt lc = {0u};
  const uint32_t lane = lane_id();
  const int wpb = SBLOCK / 64;
  const int64_t n_hard = (int64_t)rfl64(*A.n_hard);
  const int64_t n_take = n_hard < P.cap_pk ? n_hard : P.cap_pk;
  for (int64_t h = (int64_t)blockIdx.x * wpb + (int64_t)(__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6);
       h < n_take; h += (int64_t)gridDim.x * wpb) {
    const ScatItem it = scat_item(P, A, A.hard[h]);
    const double ewold = it.rec.ew / P.split2 / P.split3;
    const double thr = ewold * P.split2 * P.split1 * P.spl3_trg;
    const uint64_t key = c2d_derive_s(it.rec.key, C2D_TAG_SCAT3, it.ii, it.rec.ctr, it.rec.sub);
    for (uint32_t k0 = (uint32_t)A.sc_k1;; k0 += 64u) {
      const uint32_t k = k0 + lane;
      const bool live = k <= (uint32_t)MAX_REJECT;
      Pkt p;
      const int i_gam = scat_attempt(P, g, nel_lds, p, it.rec, key, k, ewold, live, A.kn_cap);
      const bool ok = live && (p.ew > thr || k == (uint32_t)MAX_REJECT);
      const unsigned long long m = __ballot(ok);
      if (m == 0ull) continue;
      const uint32_t kf = (uint32_t)(__ffsll((long long)m) - 1);
      {                                        /* beyond the first success: not run */
        Pkt q;
        (void)scat_attempt<-1>(P, g, nel_lds, q, it.rec, key, k, ewold, live && lane > kf, A.kn_cap);
      }
      if (lane == kf) {
        if (!(p.ew > thr)) atomicAdd(&c2d_cnt_lds[C2D_CNT_ABORTED], 1u);
        scat_emit(P, A, eic_lds, p, i_gam, ewold);
      }
      break;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C2D_NUM_NT + 2; i += SBLOCK) {
    if (nel_lds[i] != 0.0) atomicAdd(&P.T[P.off.nelectron + i], nel_lds[i]);
    if (eic_lds[i] != 0.0) atomicAdd(&P.T[P.off.E_IC + i], eic_lds[i]);
  }
  flush_counters(P, lc, lane_id());
}

/* a generation-0 source record: census packet (imcfield2d.f:98-117) or a
 * sampled volume/surface packet from the packet store.  src >= 0: the census
 * slot (the fetch resolved the chunk list once per work chunk); src < 0:
 * packet-store entry -src - 1 */
/* a census record's columns as loaded (the census branch of load_source):
 * issued by pf_issue, turned into the packet by pf_apply */
struct CensRec {
  double rpre, zpre, wmu, cphi, ew, xnu;
  uint32_t jk, bn;
  uint64_t key;
};

__device__ __forceinline__ void pf_issue(const KParams& P0, CensRec& r, long long i) {
  const KParams& P = cold(P0);
  const c2d_d2 rz = CENS_LD2(P.cin.rz + i), wp = CENS_LD2(P.cin.wp + i), ex = CENS_LD2(P.cin.ex + i);
  const c2d_u4 tg = CENS_LD4(P.cin.tg + i);
  r.rpre = rz.x; r.zpre = rz.y;
  r.wmu = wp.x; r.cphi = wp.y;
  r.ew = ex.x; r.xnu = ex.y;
  r.jk = tg.x; r.bn = tg.y;
  r.key = c2d_tg_key(tg);
}

__device__ __forceinline__ void pf_apply(const KParams& P0, Pkt& p, const CensRec& r) {
  const KParams& P = cold(P0);
  p.rpre = r.rpre; p.zpre = r.zpre;
  p.wmu = clampd(r.wmu, P.cens_wlim);               /* imcfield2d.f:119-120 (2012-11: +-1) */
  p.ew = r.ew; p.xnu = r.xnu;
#if C2D_TABLE_COMTOT
  p.eta = r.cphi;                                    /* encoded azimuth (CensusSoA) */
  p.esw = (r.bn & C2D_CENS_ESW) ? -1 : 1;
  p.phi = 0.0;
#else
  p.phi = r.cphi;
#endif
  p.jph = c2d_cens_j(r.jk); p.kph = c2d_cens_k(r.jk);
  p.ie = c2d_cens_ie(r.jk) | ((c2d_cens_efl(r.jk) + 1) << 16);   /* the bins the record carries */
  p.bins = r.bn & 0x00ffffffu;                       /* kap = 0 (census phase, H3) */
  p.key = r.key;
  p.sub = 0;
  p.dcen = P.cdt;                                    /* imcfield2d.f:117 */
  if (r.bn & C2D_CENS_VOL) p.dcen = P.cdt * c2d_draw_s(r.key, 0u, 0u);   /* vol_source's first draw */
}

/* C2D_PF_LDS: the prefetched record goes straight to LDS (gfx950 global ->
 * LDS loads, no VGPRs held while it is in flight): 16 dwords per lane in a
 * wave-private staging area, read back when the source starts */
#ifndef C2D_PF_LDS
#define C2D_PF_LDS 0
#endif
#if C2D_PF_LDS
__shared__ uint32_t c2d_pf_lds[C2D_TR_BLOCK / 64][16][64];
typedef const __attribute__((address_space(1))) void* c2d_gptr_t;
typedef __attribute__((address_space(3))) void* c2d_lptr_t;
__device__ __forceinline__ void pf_dword(const void* src, int w, int f) {
  __builtin_amdgcn_global_load_lds((c2d_gptr_t)src, (c2d_lptr_t)&c2d_pf_lds[w][f][0], 4, 0, 0);
}
__device__ __forceinline__ void pf_issue_lds(const KParams& P0, long long i) {
  const KParams& P = cold(P0);
  const int w = (int)(threadIdx.x >> 6);
  /* dwords 0-3 (rpre, zpre), 4-7 (wmu, phi), 8-11 (ew, xnu), 12-15 (jk, bins, key) */
  const uint32_t* d[4] = {reinterpret_cast<const uint32_t*>(P.cin.rz + i),
                          reinterpret_cast<const uint32_t*>(P.cin.wp + i),
                          reinterpret_cast<const uint32_t*>(P.cin.ex + i),
                          reinterpret_cast<const uint32_t*>(P.cin.tg + i)};
#pragma unroll
  for (int f = 0; f < 16; f++) pf_dword(d[f >> 2] + (f & 3), w, f);
}
__device__ __forceinline__ void pf_read_lds(CensRec& r) {
  /* the loads' LDS writes complete in vmcnt order: wait for all of them */
  __builtin_amdgcn_s_waitcnt(0xF70);                 /* vmcnt(0) */
  const int w = (int)(threadIdx.x >> 6), l = (int)(threadIdx.x & 63);
  auto dbl = [&](int f) {
    return __hiloint2double((int)c2d_pf_lds[w][2 * f + 1][l], (int)c2d_pf_lds[w][2 * f][l]);
  };
  r.rpre = dbl(0); r.zpre = dbl(1); r.wmu = dbl(2); r.cphi = dbl(3); r.ew = dbl(4); r.xnu = dbl(5);
  r.jk = c2d_pf_lds[w][12][l];
  r.bn = c2d_pf_lds[w][13][l];
  r.key = ((uint64_t)c2d_pf_lds[w][15][l] << 32) | (uint64_t)c2d_pf_lds[w][14][l];
}
#endif

__device__ __forceinline__ void load_source(const KParams& P0, Pkt& p, long long src) {
  const KParams& P = cold(P0);
  if (src >= 0) {
    CensRec r;
    pf_issue(P, r, src);
    pf_apply(P, p, r);
  } else {
    load_pk(p, P.pk, -src - 1);
    set_phi(p, p.phi);
  }
}

/* ------------------------------------------------------------------ */
/* the transport kernel: scatter secondaries of generations >= 1         */
/* ------------------------------------------------------------------ */
/* Every secondary is an imctrk2d(1) track (imctrk2d.f:662-679) from the
 * packet store; generation 0 (census + sources, the split1 probes and the
 * recombined copy) runs as probe bundles (c2d_bundle_kernel below). */
template <int V12>
__global__ void __launch_bounds__(BLOCK) C2D_TR_ATTR C2D_SFX(c2d_transport_kernel)(const KParams* __restrict__ Pg,
                                                                      const GenArgs A) {
  const KParams& P = *Pg;
  double* const lds = c2d_tr_lds;
  const int tid = threadIdx.x;
  const uint32_t lane = lane_id();
  /* LDS carve-up: Geo image | cell tallies (optional) | escape tallies */
  Tal T;
  T.g = reinterpret_cast<const Geo*>(lds);
  T.cells_off = GEO_DOUBLES;
  const int n_cells_lds = P.lds_cells ? 4 * P.ncell : 0;
  T.esc_off = GEO_DOUBLES + n_cells_lds;
  const int n_esc = P.nmu * (C2D_NPHOMAX + C2D_NPHLCMAX) + 2 * P.nz + 2 * P.nr;
  double* const cells_lds = lds + T.cells_off;
  double* const esc_lds = lds + T.esc_off;
  {
    const double* gsrc = reinterpret_cast<const double*>(P.geo);
    for (int i = tid; i < GEO_DOUBLES; i += BLOCK) lds[i] = gld(gsrc + i);
    for (int i = tid; i < n_cells_lds + n_esc; i += BLOCK) cells_lds[i] = 0.0;
  }
  init_counters(c2d_cnt_lds);
  census_chunk_load(P, tid >> 6, lane);
  __syncthreads();
  const long long n_items = (long long)rfl64(*A.n_pk);

  Pkt p;
  p.mode = 1; p.bins = 0u; p.ctr = 0; p.key = 0; p.sub = 0; p.nflight = 0;
  bool busy = false;
  ComCache cc = {-1, -1, 0.0, 0.0};
  LaneCnt lc = {0u};
  long long chunk_base = 0, chunk_end = 0;
  bool exhausted = false;
  Prof pf;
#ifdef C2D_TR_PROF
  for (int i = 0; i < C2D_TR_PROF_WORDS; i++) pf.acc[i] = 0;
  pf.t = clock64();
#endif

  for (;;) {
    /* ---- refill idle lanes: chunked, wave-aggregated work fetch ---- */
    bool got = false;
    long long item = -1;
    if (!exhausted) {
      unsigned long long needm = __ballot(!busy);
      while (needm != 0ull) {
        if (chunk_base >= chunk_end) {
          unsigned long long nb = 0;
          if (lane == 0) nb = atomicAdd(A.work_counter, (unsigned long long)CHUNK);
          nb = rfl64(nb);
          if ((long long)nb >= n_items) { exhausted = true; break; }
          chunk_base = (long long)nb;
          chunk_end = chunk_base + CHUNK < n_items ? chunk_base + CHUNK : n_items;
        }
        const long long avail = chunk_end - chunk_base;
        const unsigned long long lt = (lane == 0) ? 0ull : (needm & ((~0ull) >> (64 - lane)));
        const long long rank = __popcll(lt);
        const long long nneed = __popcll(needm);
        if (((needm >> lane) & 1ull) && rank < avail) {
          item = chunk_base + rank;
          got = true;
        }
        chunk_base += (nneed < avail ? nneed : avail);
        needm = __ballot(!busy && !got);
      }
    }
    TP_MARK(pf, TP_REFILL);
#ifdef C2D_TR_PROF
    pf.acc[TP_ITER] += 1;
#endif
    if (got) {
      TP_COUNT(pf, TP_GOT_W, TP_GOT_L);
      load_pk(p, cold(P).pk, item);
      set_phi(p, p.phi);
      p.mode = 1;
      p.wtmin = 1.0e-10 * p.ew;
      p.nflight = 0;
      cc.cell0 = -1; cc.cell1 = -1;
      cache_energy(P, T.g, p);
      busy = true;
    }
    if (exhausted && __ballot(busy) == 0ull) break;
    TP_MARK(pf, TP_START);
    if (busy) {
#ifdef C2D_TR_PROF
      pf.acc[TP_LANES] += __popcll(__ballot(1));
#endif
      const int out = flight<V12>(P, T, p, cc, lc, pf);
      TP_MARK(pf, TP_EVENT);
      if (out != FL_CONT) {
        if (out == FL_COLLIDE) push_scat(P, A.q2_out, A.n2_out, make_rec(p, p.key, p.ctr));
        busy = false;
      }
    }
    TP_MARK(pf, TP_POST);
  }
#ifdef C2D_TR_PROF
  pf.acc[TP_NWAVE] = 1;
  if (lane == 0)
    for (int i = 0; i < C2D_TR_PROF_WORDS; i++)
      if (pf.acc[i]) atomicAdd(&P.prof[i], (unsigned long long)pf.acc[i]);
#endif
  census_chunk_store(P, tid >> 6, lane);

  /* ---- flush: LDS tallies and counters ---- */
  __syncthreads();
  if (P.lds_cells) {
    double* gdst = P.T + P.off.edep;    /* edep, prdep, ecens, npcen are contiguous */
    for (int i = tid; i < n_cells_lds; i += BLOCK) {
      double v = cells_lds[i];
      if (v != 0.0) atomicAdd(&gdst[i], v);
    }
  }
  {
    double* gdst = P.T + P.off.fout;    /* fout, edout, erlki, erlko, erlku, erlkl */
    for (int i = tid; i < n_esc; i += BLOCK) {
      double v = esc_lds[i];
      if (v != 0.0) atomicAdd(&gdst[i], v);
    }
  }
  lc.paths = lc.steps;                  /* per-copy tracking: one copy per path */
  flush_counters(P, lc, lane);
}

/* ------------------------------------------------------------------ */
/* generation 0 as probe bundles                                        */
/* ------------------------------------------------------------------ */
/* The split1 probe copies of a source (imctrk2d(-1), imctrk2d.f:106-123)
 * and its recombined copy (imctrk2d(0), :690-704) start from the same
 * record and differ only in weight and random numbers: they fly the same
 * path until a probe collides.  A bundle carries up to BUNDLE_MAX probes
 * and the recombined copy along one shared path: comtot, the geometry, the
 * absorption factor and the position update are evaluated once per shared
 * step.
 *
 * Collisions: each probe's collision process along the path has the same
 * rate sigsc, so (superposition) the first collision among the n probes on
 * the path comes after an optical depth tau ~ Exp(n) per probe, the collider
 * is uniform among the n, and by memorylessness the others fly on unchanged
 * -- the per-copy tracker's process (a fresh colmfp per copy and step,
 * imctrk2d.f:150-160) with other random numbers.  The bundle draws from its
 * own stream (source key, C2D_SUB_BUNDLE | g0): tau at the start; per
 * collision the collider, its absorption point, the others' new tau; per
 * step the survivors' absorption points (only where xabs > 1e-5) in probe
 * order.  A step needs no random number unless a probe collides in it or
 * absorption is sampled.  The collider leaves through its own partial step
 * (flight()'s ikind = 3 branch) and its collision record carries its own
 * sub-stream (source key, 1 + probe).  The oracle's lineage mode tracks
 * probes the same way (oracle/c2d_oracle.c probe_bundle); DESIGN.md §2c.
 *
 * The recombined copy's weight (split1 - nscat) * s_ew needs the source's
 * final collision count, so it flies with the bundle of the last probes on
 * the assumption that they do not collide; a collision in that bundle
 * cancels it (the packet-steps it was counted for are taken back) and it
 * flies alone from the source afterwards.  Its absorption-point draws are
 * only counted (its prdep is never tallied).  Geometry, absorption,
 * deposits, records and counters are the per-copy tracker's; the cell
 * tallies are summed in another order. */
constexpr int BUNDLE_MAX = 32;
/* C2D_PF_SRC: each lane claims its next census source while it runs the
 * current one and issues that record's loads after the step's table loads
 * have been waited for, so they complete under the rest of the step instead
 * of stalling the next bundle_begin (packet-store sources load as before) */
#ifndef C2D_PF_SRC
#define C2D_PF_SRC 1
#endif
enum : int32_t {
  BF_TRACK = 1,     /* the recombined copy is on the path               */
  BF_SPEC = 2,      /* ... with a weight that assumes no more collisions */
  BF_RERUN = 4,     /* a collision cancelled it: refly alone afterwards  */
  BF_TKILL = 8,     /* it ended KILLED / ABORTED: counted at the bundle end */
  BF_TABORT = 16
};
struct Bundle {
  Pkt p;              /* shared path; p.ew, p.wtmin, p.ctr: the recombined copy's */
  double ewp, wtminp; /* the probes' common weight and kill threshold               */
  double tau;         /* optical depth (per probe) to the next collision among them */
  long long src;      /* source item                                             */
  uint32_t alive;     /* probes g0 + i still on the path (bit i)                 */
  uint32_t bctr;      /* draws consumed from the bundle stream                   */
  uint32_t actr;      /* outputs consumed from the absorption-point stream       */
  int32_t g0;         /* first probe of this bundle (== split1: refly alone)     */
  int32_t nscat;      /* probes of the source that collided                      */
  int32_t flags;
  int32_t tsteps;     /* packet-steps counted for a speculative recombined copy  */
};

/* next draw of the bundle stream (source key, C2D_SUB_BUNDLE | g0) */
__device__ __forceinline__ double UB(Bundle& b) {
  return c2d_draw_s(b.p.key, C2D_SUB_BUNDLE | (uint32_t)b.g0, b.bctr++);
}

/* start (or restart) the bundle at probe g0 of source b.src */
__device__ __forceinline__ void bundle_begin(const KParams& P, const Tal& T, Bundle& b,
                                             bool from_pf = false, const CensRec* pr = nullptr) {
  Pkt& p = b.p;
#if C2D_PF_LDS
  (void)pr;
  if (from_pf) {                      /* the census record prefetched into LDS */
    CensRec r;
    pf_read_lds(r);
    pf_apply(P, p, r);
  } else {
    load_source(P, p, b.src);
  }
#else
  if (from_pf) pf_apply(P, p, *pr);   /* the census record prefetched into pr */
  else load_source(P, p, b.src);
#endif
  const double ew0 = p.ew;
  const double s_ew = FDIV_POS(ew0, (double)P.split1);   /* imctrk2d.f:106-123 */
  const int G = min(P.split1 - b.g0, BUNDLE_MAX);
  b.ewp = s_ew;
  b.wtminp = 1.0e-10 * ew0;
  b.alive = G >= 32 ? 0xffffffffu : ((1u << G) - 1u);
  b.bctr = 0;
  b.actr = 0;
  b.flags = 0;
  b.tsteps = 0;
  b.tau = 0.0;
  if (G > 0) b.tau = FDIV_POS(-TAU_LOG(UB(b)), (double)G);
  p.nflight = 0;
  p.mode = 0;
  if (b.g0 + G == P.split1 && P.split1 - b.nscat > 0) {
    /* recombined unscattered copies, imctrk2d(0) (imctrk2d.f:690-704) */
    p.ew = (double)(P.split1 - b.nscat) * s_ew;
    p.wtmin = 1.0e-10 * p.ew;
    p.sub = C2D_SUB_RECOMB;
    p.ctr = 0;
    b.flags = BF_TRACK | (G > 0 ? BF_SPEC : 0);
  }
  cache_energy(P, T.g, p, b.src >= 0);   /* census records carry ie; azimuth: set by load_source */
}

/* probe g0 + i collides at dcol inside the shared step: its own partial
 * step to the collision point (flight(), ikind = 3), then the record */
template <int V12>
__device__ __forceinline__ void probe_collide(const KParams& P, const Tal& T, const GenArgs& A,
                                              Bundle& b, int i, double dcol, double sigabs,
                                              double Eta, double swmu, int eta_switch, int cell,
                                              LaneCnt& lc) {
  const double lim9 = V12 ? 1.0 : 0.999999999;
  const Pkt& p = b.p;
  const double rpre = p.rpre, zpre = p.zpre, wmu = p.wmu;
  const double trld = dcol;
  const double f = trld * swmu;
  const double rnew = FSQRT(f * f + rpre * rpre + 2.0 * f * rpre * Eta);
  const double znew = zpre + trld * wmu;
  const double xabs = sigabs * trld;
  const double ewnew = (xabs < 100.0) ? b.ewp * FEXP(-xabs) : 0.0;
  double deleabs = b.ewp - ewnew;
  if (deleabs < 1.0e-50) deleabs = 1.0e-50;
  double wmustar;
  if (xabs <= 0.00001) {
    wmustar = wmu;
  } else {
    /* one draw: mr < 1 <= ew / deleabs always holds (ew >= 1e-40) */
    const double mr = UB(b);
    const double sstar = FDIV_POS(-FLOG(1.0 - FDIV_POS(mr * deleabs, b.ewp)), sigabs);
    const double denom = FSQRT(rpre * rpre + 2.0 * wmu * rpre * sstar + sstar * sstar);
    wmustar = FDIV_POS(wmu * rpre + sstar, denom);
  }
  cell_add(P, T, TC_EDEP, cell, deleabs);
  cell_add(P, T, TC_PRDEP, cell, deleabs * wmustar * C_LIGHT);
  if (ewnew <= b.wtminp) {
    LC_ADD(lc, C2D_CNT_KILLED);
    return;
  }
  LC_ADD(lc, C2D_CNT_COLLIDE);
  double Eta2 = clampd(FDIV_NN((V12 ? f : trld) + Eta * rpre, rnew), lim9);   /* H1 unless 2012-11 */
  double phi = c2d_acos(Eta2);
  if (eta_switch == -1) phi = 2.0 * PI_REF - phi;
  ScatRec r;
  r.rpre = rnew; r.zpre = znew; r.wmu = wmu; r.phi = phi; r.ew = ewnew; r.xnu = p.xnu;
  r.dcen = p.dcen - trld;
  r.jk = ((uint32_t)p.jph << 16) | (uint32_t)p.kph;
  r.ctr = b.bctr;
  r.key = p.key;
  r.kap = (uint32_t)KAP(p);
  r.sub = 1u + (uint32_t)(b.g0 + i);
  push_scat(P, A.q2_out, A.n2_out, r);
  b.nscat++;
  if (b.flags & BF_SPEC) {
    /* the recombined copy's weight assumed no collision: cancel it, and the
     * packet-steps it was counted for (it may have ended already) */
    lc.steps -= (uint32_t)b.tsteps;
    b.flags = (b.flags & ~(BF_TRACK | BF_SPEC | BF_TKILL | BF_TABORT)) | BF_RERUN;
  }
}

/* one shared step of the bundle (flight() for every copy on the path) */
template <int V12>
__device__ __forceinline__ void bundle_step(const KParams& P1, const Tal& T, const GenArgs& A,
                                            Bundle& b, ComCache& cc, LaneCnt& lc, Prof& pf,
                                            CensRec& nr, long long nitem, int& nst) {
#ifdef C2D_HOT_RELOAD
  const KParams& P = cold_always(P1);
#else
  const KParams& P = P1;
#endif
  const double lim8 = V12 ? 1.0 : 9.9999999e-1, lim9 = V12 ? 1.0 : 0.999999999;
  const Geo* g = T.g;
  Pkt& p = b.p;
  if (b.alive && b.ewp < 1.0e-40) b.alive = 0;
  if ((b.flags & BF_TRACK) && p.ew < 1.0e-40) b.flags &= ~BF_TRACK;
  if (!b.alive && !(b.flags & BF_TRACK)) return;
  if (++p.nflight > MAX_FLIGHTS) {
    atomicAdd(&c2d_cnt_lds[C2D_CNT_ABORTED], (uint32_t)__popc(b.alive));
    b.alive = 0;
    if (b.flags & BF_TRACK) b.flags = (b.flags & ~BF_TRACK) | BF_TKILL | BF_TABORT;
    return;
  }
  p.wmu = clampd(p.wmu, lim8);
  lc.paths++;
  const int cell = (p.jph - 1) * P.nr + (p.kph - 1);
  /* the step's absorption coefficient: issued before the comtot lookup and
   * the geometry, used after them */
  const double kap_cell = gld((KAP(p) ? P.kappa_s : P.kappa_cv) + (int64_t)cell * C2D_N_VOL + ((p.ie & 0xffff) - 1));
  double sigsc = 1.0;
  if (b.alive) {
#if C2D_TABLE_COMTOT
    sigsc = comtot_table(P, cell, p.xnu, p.tg, p.tt);
    (void)cc;
#else
    if (cc.cell0 == cell) {
      sigsc = cc.v0;
    } else if (cc.cell1 == cell) {
      sigsc = cc.v1;
    } else {
      sigsc = comtot_exact(P, cell, p.xnu);
      cc.cell1 = cc.cell0; cc.v1 = cc.v0;
      cc.cell0 = cell; cc.v0 = sigsc;
    }
#endif
  }
  /* geometry (imctrk2d.f:228-379), shared */
  const double rkm1 = (p.kph == 1) ? P.rmin : g->r[p.kph - 1];
  const double xqsqleft = rkm1 * rkm1;
#if C2D_TABLE_COMTOT
  double Eta = p.eta;
  const int eta_switch = p.esw;
#else
  double Eta = c2d_cos(p.phi);
  const int eta_switch = (p.phi <= PI_REF && p.phi >= 1.0e-10) ? 1 : -1;
#endif
  if (!V12) Eta = clampd(Eta, lim8);
  const double rpre = p.rpre, zpre = p.zpre, wmu = p.wmu;
  const double disp = Eta * rpre;
  const double psq = rpre * rpre * (1.0 - Eta * Eta);
  int kbnd, inout, knew, jnew;
  double rbnd, Zbnd;
  if (Eta < 0.0 && psq < xqsqleft) {
    kbnd = p.kph - 1;
    inout = -1;
    rbnd = rkm1;
  } else {
    kbnd = p.kph;
    inout = 1;
    rbnd = g->r[p.kph];
  }
  double dpbsq = rbnd * rbnd - psq;
  if (dpbsq < 1.0e-6) dpbsq = 1.0e-6;
  const double disbr = (double)inout * FSQRT(dpbsq) - disp;
  const double swmu = FSQRT(1.0 - wmu * wmu);
  double trldb = FDIV_POS(disbr, swmu);
  double fr = disbr;                    /* V12: the reference's f on a boundary step */
  const double Zr = zpre + wmu * trldb;
  const double zlow = (p.jph == 1) ? P.zmin : g->z[p.jph - 1];
  const double zup = g->z[p.jph];
  if (Zr > zup || Zr < zlow) {
    Zbnd = (Zr > zup) ? zup : zlow;
    knew = p.kph;
    jnew = (Zr > zup) ? p.jph + 1 : p.jph - 1;
    const double f = FDIV_POS((Zbnd - zpre) * swmu, wmu);   /* wmu != 0 on a z crossing */
    fr = f;
    rbnd = FSQRT(rpre * rpre + f * f + 2.0 * rpre * f * Eta);
    trldb = FSQRT(f * f + (Zbnd - zpre) * (Zbnd - zpre));
  } else {
    knew = p.kph + inout;
    jnew = p.jph;
    rbnd = (kbnd > 0) ? g->r[kbnd] : P.rmin;
    Zbnd = Zr;
  }
  /* every copy that does not collide: boundary if trldb < dcen, else census */
  const bool bnd = trldb < p.dcen;
  const double trld = bnd ? trldb : p.dcen;
  double sigabs = 1.0e-40 + 1.0 * kap_cell;
  if (sigabs < 1.0e-40) sigabs = 1.0e-40;
  const double xabs = sigabs * trld;
  const double ex = (xabs < 100.0) ? FEXP(-xabs) : 0.0;
  const bool two = xabs > 0.00001;      /* the absorption point is sampled */
  TP_MARK(pf, TP_GEOM);
  /* ---- probes (mode -1): collisions and weights; their absorption-point
   * deposits are deferred to the end of the step (below) ---- */
  int nabs = 0;                 /* survivors that deposit over the whole step */
  double dabs = 0.0, qabs = 0.0;
  if (b.alive) {
    int n = __popc(b.alive);
    lc.steps += (uint32_t)n;
    /* collisions inside the step (ikind 3: dcol < dcen, not trldb < dcol) */
    double dpos = 0.0;
    for (;;) {
      const double dcol = dpos + FDIV_POS(b.tau, sigsc);
      if (!(dcol < p.dcen && !(trldb < dcol))) break;
      int k = (int)(UB(b) * (double)n);
      if (k > n - 1) k = n - 1;
      uint32_t m = b.alive;
      for (; k > 0; k--) m &= m - 1u;
      const int i = __ffs(m) - 1;
      b.alive &= ~(1u << i);
      n--;
      probe_collide<V12>(P, T, A, b, i, dcol, sigabs, Eta, swmu, eta_switch, cell, lc);
      dpos = dcol;
      if (n == 0) break;
      b.tau = FDIV_POS(-TAU_LOG(UB(b)), (double)n);
    }
    if (n > 0) {
      b.tau = b.tau - sigsc * (trld - dpos);
      /* the n probes that fly the whole step (imctrk2d.f:382-462) */
      const double ewnew = (xabs < 100.0) ? b.ewp * ex : 0.0;
      double deleabs = b.ewp - ewnew;
      if (deleabs < 1.0e-50) deleabs = 1.0e-50;
      nabs = n;
      dabs = deleabs;
      qabs = FDIV_POS(deleabs, b.ewp);
      if (ewnew <= b.wtminp) {
        atomicAdd(&c2d_cnt_lds[C2D_CNT_KILLED], (uint32_t)n);
        b.alive = 0;
      } else {
        b.ewp = ewnew;
      }
    }
  }
  TP_MARK(pf, TP_ABS);
  /* ---- the recombined copy (mode 0) ---- */
  if (b.flags & BF_TRACK) {
    lc.steps++;
    if (b.flags & BF_SPEC) b.tsteps++;
    const double ewnew = (xabs < 100.0) ? p.ew * ex : 0.0;
    if (two) p.ctr++;                 /* its absorption-point draw: prdep is not tallied */
    if (ewnew <= p.wtmin) b.flags = (b.flags & ~BF_TRACK) | BF_TKILL;
    else p.ew = ewnew;
  }
  /* ---- the shared move and the recombined copy's event.  Census records
   * and escape events are stored here, before the survivors' point loop:
   * stores and the n_field atomic count in vmcnt with the loads, so the
   * VALU-only loop below lets them drain before the next load is waited
   * for. ---- */
  if (b.alive || (b.flags & BF_TRACK)) {
    double rnew, znew;
    if (bnd) {
      rnew = rbnd;
      znew = Zbnd;
    } else {
      jnew = p.jph;
      knew = p.kph;
      const double f = trld * swmu;
      fr = f;
      rnew = FSQRT(f * f + rpre * rpre + 2.0 * f * rpre * Eta);
      znew = zpre + trld * wmu;
    }
    p.dcen = p.dcen - trld;
    /* hazard H1: trld, not f (imctrk2d.f:472); f in src_20121113:478 */
    double Etan = FDIV_NN((V12 ? fr : trld) + Eta * rpre, rnew);
    Etan = clampd(Etan, lim9);
    const bool leaves = bnd && (jnew == P.nz + 1 || jnew == 0 || knew == P.nr + 1 || knew == 0);
#if C2D_TABLE_COMTOT
    p.eta = Etan;
    if ((b.flags & BF_TRACK) && leaves) {   /* an escape event reads phi (census: encoded) */
      p.phi = c2d_acos(Etan);
      if (eta_switch == -1) p.phi = 2.0 * PI_REF - p.phi;
    }
#else
    p.phi = c2d_acos(Etan);
    if (eta_switch == -1) p.phi = 2.0 * PI_REF - p.phi;
#endif
    p.rpre = rnew;
    p.zpre = znew;
    TP_MARK(pf, TP_EVENT);
    if (bnd) {
      if (leaves) {
        b.alive = 0;                            /* probes leaving end (no tally) */
        p.jph = jnew;
        p.kph = knew;
        if (b.flags & BF_TRACK) {
          TP_COUNT(pf, TP_LEAK_W, TP_LEAK_L);
          if (imcleak(P, T, p, lc) == 1) b.flags &= ~BF_TRACK;
          else set_phi(p, p.phi);               /* axis pass-through set phi = 1e-6 */
        }
      } else {
        p.kph = knew;
        p.jph = jnew;
      }
    } else {
      /* census (imctrk2d.f:528-578): probes end, the recombined copy is written */
      b.alive = 0;
      if (b.flags & BF_TRACK) {
        TP_COUNT(pf, TP_CENS_W, TP_CENS_L);
        census_write(P, T, p, lc);
        b.flags &= ~BF_TRACK;
      }
    }
    TP_MARK(pf, TP_CWR);
  }
  /* ---- the survivors' absorption points and deposits (imctrk2d.f:382-462),
   * at the step's starting point ---- */
  TP_MARK(pf, TP_EVENT);
#if C2D_PF_SRC
  /* the step's own loads have been waited for and its records stored: the
   * next source's record loads issue here and complete under the VALU-only
   * point loop and the refill */
  if (nst == 1 && nitem >= 0) {
#if C2D_PF_LDS
    pf_issue_lds(P, nitem);
    (void)nr;
#else
    pf_issue(P, nr, nitem);
#endif
    nst = 2;
  }
#else
  (void)nr; (void)nitem; (void)nst;
#endif
  if (nabs > 0) {
    double sum_prdep = 0.0;
#ifdef C2D_ABLATE_PROBE_ABS            /* profiling ablation only (tools/build_sweep.sh) */
    if (two && nabs < 0) {
#else
    if (two) {
#endif
      /* two 32-bit uniforms per output of the bundle's point stream
       * (c2d_abspt), fresh outputs per shared step */
      const uint32_t sub = C2D_SUB_ABSPT | (uint32_t)b.g0;
#if C2D_TABLE_COMTOT && C2D_PT_F32
      /* wmustar = (wmu*rpre + s) / |r + s d| with |r + s d|^2 written as
       * (s + wmu*rpre)^2 + rpre^2 (1 - wmu^2): a sum of non-negative terms,
       * no cancellation near the axis in f32.  u: the top 24 bits of each
       * 32-bit half of the point stream's output, (u + 1/2) 2^-24 in (0,1)
       * exactly in f32; -log(1-x) by its series below 1e-2 (truncation
       * < x^4/5), else by v_log_f32.  Lengths in units of rs = max(rpre,
       * 1/sigabs) (wmustar is a ratio of lengths): s/rs, rpre/rs <= O(10),
       * so nothing overflows f32 however large rpre (1.8e19 cm unscaled) */
      {
        const double sr = sigabs * rpre;            /* rpre in absorption lengths */
        const double a = sr < 1.0 ? sr : 1.0;       /* rpre / rs */
        const float isig = (float)(sr > 1.0 ? FDIV_POS(1.0, sr) : 1.0);   /* 1 / (sigabs rs) */
        const float Aw = (float)(wmu * a);
        const float Cw = (float)(a * a * (1.0 - wmu * wmu));
        const float qf = (float)qabs;
        float wsum = 0.0f;
        /* c2d_abspt(key, sub, n) = mix64(key + gamma ((sub << 32 | n) + 1)):
         * the argument advances by gamma per output (an add, not a 64-bit
         * multiply per output); the same outputs */
        uint64_t zst = p.key + 0x9E3779B97F4A7C15ull * ((((uint64_t)sub << 32) | (uint64_t)b.actr) + 1ull);
        for (int t = 0; t < nabs; t += 2) {
          const uint64_t wo = c2d_mix64(zst);
          zst += 0x9E3779B97F4A7C15ull;
          b.actr++;
#pragma unroll
          for (int j = 0; j < 2; j++) {
            if (t + j < nabs) {
              const uint32_t u = j == 0 ? (uint32_t)(wo >> 32) : (uint32_t)wo;
              /* the top 24 bits by one v_cvt_f32_u32: written as (float)(u >> 8),
               * the high half's conversion was widened to a 64-bit shift and a
               * u64 -> f32 expansion (7 more instructions) */
              float fu;
              __asm__("v_cvt_f32_u32 %0, %1" : "=v"(fu) : "v"(u >> 8));
              const float x = (fu + 0.5f) * (5.9604644775390625e-8f * qf);
              const float L = (x < 1.0e-2f)
                  ? x * __builtin_fmaf(x, __builtin_fmaf(x, __builtin_fmaf(x, 0.25f, 0.33333334f), 0.5f), 1.0f)
                  : -0.69314718f * __builtin_amdgcn_logf(1.0f - x);
              const float tt = __builtin_fmaf(L, isig, Aw);          /* s + wmu*rpre */
              wsum += tt * __builtin_amdgcn_rsqf(__builtin_fmaf(tt, tt, Cw));
            }
          }
        }
        sum_prdep = dabs * (double)wsum * C_LIGHT;
      }
#else
#if C2D_TABLE_COMTOT
      const double isig = FDIV_POS(1.0, sigabs);
      const double Aw = wmu * rpre, Bw = rpre * rpre;
#endif
#if C2D_TABLE_COMTOT
      /* -log(1-x) for x = u * qabs: the series below 1e-2 (8 terms, truncation
       * < x^8/9 relative; 1e-4 with 4 terms -3 %, 0.05 with 12 terms or
       * 2 atanh(x/(2-x)) below 0.2: no better, r02ap-aq; 4 terms in waves
       * whose every qabs < 1e-4: +-0, r03u), else the log */
#define C2D_PT_LOOP(LEXPR)                                                               \
      for (int t = 0; t < nabs; t += 2) {                                                \
        const uint64_t wo = c2d_abspt(p.key, sub, b.actr++);                             \
        _Pragma("unroll") for (int j = 0; j < 2; j++) {                                  \
          if (t + j < nabs) {                                                            \
            const double x = c2d_u01_32(j == 0 ? (uint32_t)(wo >> 32) : (uint32_t)wo) * qabs; \
            const double L = (LEXPR);                                                    \
            const double sstar = L * isig;                                               \
            /* 1/sqrt(d) from v_rsq_f64 and two Newton steps (f64 accurate) */           \
            const double d = Bw + sstar * (2.0 * Aw + sstar);                            \
            const double h = 0.5 * d;                                                    \
            double y = __builtin_amdgcn_rsq(d);                                          \
            _Pragma("unroll") for (int nr = 0; nr < C2D_RSQ_NR; nr++)                    \
              y = y * __builtin_fma(-h, y * y, 1.5);                                     \
            sum_prdep += dabs * ((Aw + sstar) * y) * C_LIGHT;                            \
          }                                                                              \
        }                                                                                \
      }
#if C2D_PT_SERIES
      C2D_PT_LOOP((x < 1.0e-2)
          ? x * C2D_MADD(x, C2D_MADD(x, C2D_MADD(x, C2D_MADD(x, C2D_MADD(x, C2D_MADD(x,
                C2D_MADD(x, 0.125, 0.14285714285714286), 0.16666666666666667), 0.2), 0.25),
                0.33333333333333333), 0.5), 1.0)
          : -FLOG(1.0 - x));
#else
      C2D_PT_LOOP(-FLOG(1.0 - x));
#endif
#undef C2D_PT_LOOP
#else
      for (int t = 0; t < nabs; t += 2) {
        const uint64_t wo = c2d_abspt(p.key, sub, b.actr++);
#pragma unroll
        for (int j = 0; j < 2; j++) {
          if (t + j < nabs) {
            const double x = c2d_u01_32(j == 0 ? (uint32_t)(wo >> 32) : (uint32_t)wo) * qabs;
            const double sstar = -c2d_log_pos(1.0 - x) / sigabs;
            const double denom = FSQRT(rpre * rpre + 2.0 * wmu * rpre * sstar + sstar * sstar);
            sum_prdep += dabs * ((wmu * rpre + sstar) / denom) * C_LIGHT;
          }
        }
      }
#endif
#endif   /* C2D_PT_F32 */
    } else {
      sum_prdep = (double)nabs * (dabs * wmu * C_LIGHT);
    }
    cell_add(P, T, TC_EDEP, cell, (double)nabs * dabs);
    cell_add(P, T, TC_PRDEP, cell, sum_prdep);
  }
  TP_MARK(pf, TP_PTS);
}

template <int V12>
__global__ void __launch_bounds__(BLOCK) C2D_TR_ATTR C2D_SFX(c2d_bundle_kernel)(const KParams* __restrict__ Pg,
                                                                   const GenArgs A) {
  const KParams& P = *Pg;
  double* const lds = c2d_tr_lds;
  const int tid = threadIdx.x;
  const uint32_t lane = lane_id();
  Tal T;
  T.g = reinterpret_cast<const Geo*>(lds);
  T.cells_off = GEO_DOUBLES;
  const int n_cells_lds = P.lds_cells ? 4 * P.ncell : 0;
  T.esc_off = GEO_DOUBLES + n_cells_lds;
  const int n_esc = P.nmu * (C2D_NPHOMAX + C2D_NPHLCMAX) + 2 * P.nz + 2 * P.nr;
  double* const cells_lds = lds + T.cells_off;
  double* const esc_lds = lds + T.esc_off;
  {
    const double* gsrc = reinterpret_cast<const double*>(P.geo);
    for (int i = tid; i < GEO_DOUBLES; i += BLOCK) lds[i] = gld(gsrc + i);
    for (int i = tid; i < n_cells_lds + n_esc; i += BLOCK) cells_lds[i] = 0.0;
  }
  init_counters(c2d_cnt_lds);
  __syncthreads();
  const long long n_items = (long long)A.n_items;

  Bundle b;
  b.p.mode = 0; b.p.bins = 0u; b.p.ctr = 0; b.p.key = 0; b.p.sub = 0; b.p.nflight = 0;
  b.alive = 0; b.flags = 0; b.src = 0; b.g0 = 0; b.nscat = 0; b.bctr = 0; b.tsteps = 0;
  b.tau = 0.0; b.ewp = 0.0; b.wtminp = 0.0;
  bool busy = false;
  ComCache cc = {-1, -1, 0.0, 0.0};
  LaneCnt lc = {0u};
  long long chunk_base = 0, chunk_end = 0;
  long long chunk_slot = 0;        /* census slot of the work chunk's first item */
  bool exhausted = false;
  int shard_try = 0;
  const int shard0 = (int)(blockIdx.x % C2D_WORK_SHARDS);
  Prof pf;
#ifdef C2D_TR_PROF
  for (int i = 0; i < C2D_TR_PROF_WORDS; i++) pf.acc[i] = 0;
  pf.t = clock64();
#endif
  census_chunk_load(P, tid >> 6, lane);
  /* the lane's next source (C2D_PF_SRC): nst 0 none, 1 claimed, 2 record loaded */
  CensRec nr = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0u, 0u, 0ull};
  long long nitem = 0;
  int nst = 0;

  /* chunked, wave-aggregated work fetch from the workgroup's shard of the
   * item range, then from the following ones: every lane with `want` gets
   * the next item (its census slot or packet-store entry) while items last */
  auto claim = [&](bool want, long long& it_out) -> bool {
    bool ok = false;
    unsigned long long needm = __ballot(want);
    while (needm != 0ull) {
      if (chunk_base >= chunk_end) {
        for (;;) {
          if (shard_try >= C2D_WORK_SHARDS) { exhausted = true; break; }
          /* shard bounds on work-chunk (= census-chunk) boundaries */
          const int s = (shard0 + shard_try) % C2D_WORK_SHARDS;
          const long long lo = (n_items * s / C2D_WORK_SHARDS) & ~(CHUNK - 1);
          const long long hi = s + 1 == C2D_WORK_SHARDS
                                   ? n_items : (n_items * (s + 1) / C2D_WORK_SHARDS) & ~(CHUNK - 1);
          unsigned long long nb = 0;
          if (lane == 0)
            nb = atomicAdd(A.work_sh + (size_t)s * C2D_EV_SHARD_STRIDE, (unsigned long long)CHUNK);
          nb = rfl64(nb);
          if (lo + (long long)nb < hi) {
            chunk_base = lo + (long long)nb;
            chunk_end = chunk_base + CHUNK < hi ? chunk_base + CHUNK : hi;
            chunk_slot = chunk_base;
            if (cold(P).clist && chunk_base < cold(P).n_cens_items) {
              const int32_t id = __builtin_amdgcn_readfirstlane(gld(cold(P).clist + (chunk_base >> C2D_CCHUNK_LOG)));
              chunk_slot = (long long)id << C2D_CCHUNK_LOG;
              if (lane == 0)
                census_track(tid >> 6, id,
                             (uint32_t)(min(chunk_end, (long long)cold(P).n_cens_items) - chunk_base));
            }
            break;
          }
          shard_try++;
        }
        if (exhausted) break;
      }
      const long long avail = chunk_end - chunk_base;
      const unsigned long long lt = (lane == 0) ? 0ull : (needm & ((~0ull) >> (64 - lane)));
      const long long rank = __popcll(lt);
      const long long nneed = __popcll(needm);
      if (((needm >> lane) & 1ull) && rank < avail) {
        const long long it = chunk_base + rank;
        it_out = it < cold(P).n_cens_items ? chunk_slot + (it & (CHUNK - 1))
                                           : -(it - cold(P).n_cens_items) - 1;
        ok = true;
      }
      chunk_base += (nneed < avail ? nneed : avail);
      needm = __ballot(want && !ok);
    }
    return ok;
  };

  for (;;) {
    /* ---- refill idle lanes: the prefetched source, else a fetched one;
     * then claim the next source of every lane that has none ---- */
    bool got = false, from_pf = false;
    long long item = -1;
#if C2D_PF_SRC
    if (!busy && nst != 0) {
      got = true;
      item = nitem;
      from_pf = nst == 2;
      nst = 0;
    }
#endif
    if (!exhausted) {
      const bool g2 = claim(!busy && !got, item);
      got = got || g2;
    }
#if C2D_PF_SRC
    if (!exhausted) {
      long long ni = 0;
      if (claim((busy || got) && nst == 0, ni)) {
        nitem = ni;
        nst = 1;
      }
    }
#endif
    TP_MARK(pf, TP_REFILL);
#ifdef C2D_TR_PROF
    pf.acc[TP_ITER] += 1;
#endif
    if (got) {
      TP_COUNT(pf, TP_GOT_W, TP_GOT_L);
      LC_ADD(lc, C2D_CNT_SOURCES);      /* imctrk2d(-1) entry (imctrk2d.f:91,106-123) */
      b.src = item;
      b.g0 = 0;
      b.nscat = 0;
      cc.cell0 = -1; cc.cell1 = -1;
      bundle_begin(P, T, b, from_pf, &nr);
      busy = true;
    }
    if (exhausted && __ballot(busy) == 0ull) break;
    TP_MARK(pf, TP_START);
    if (busy) {
#ifdef C2D_TR_PROF
      pf.acc[TP_LANES] += __popcll(__ballot(1));
#endif
      bundle_step<V12>(P, T, A, b, cc, lc, pf, nr, nitem, nst);
      TP_MARK(pf, TP_EVENT);
      if (!b.alive && !(b.flags & BF_TRACK)) {
        if ((b.flags & (BF_TKILL | BF_RERUN)) == BF_TKILL)
          LC_ADD(lc, (b.flags & BF_TABORT) ? C2D_CNT_ABORTED : C2D_CNT_KILLED);
        const int G = min(P.split1 - b.g0, BUNDLE_MAX);
        if (b.g0 + G < P.split1) {
          TP_COUNT(pf, TP_RST_W, TP_RST_L);
          b.g0 += G;                        /* next bundle of probes */
          bundle_begin(P, T, b);
        } else if ((b.flags & BF_RERUN) && P.split1 - b.nscat > 0) {
          TP_COUNT(pf, TP_RST_W, TP_RST_L);
          b.g0 = P.split1;                  /* the recombined copy alone */
          bundle_begin(P, T, b);
        } else {
          busy = false;
          if (cold(P).clist && b.src >= 0) census_item_done(P, b.src);
        }
      }
    }
    TP_MARK(pf, TP_POST);
  }
#ifdef C2D_TR_PROF
  pf.acc[TP_NWAVE] = 1;
  if (lane == 0)
    for (int i = 0; i < C2D_TR_PROF_WORDS; i++)
      if (pf.acc[i]) atomicAdd(&P.prof[i], (unsigned long long)pf.acc[i]);
#endif

  census_chunk_store(P, tid >> 6, lane);

  /* ---- flush: LDS tallies and counters ---- */
  __syncthreads();
  if (P.lds_cells) {
    double* gdst = P.T + P.off.edep;
    for (int i = tid; i < n_cells_lds; i += BLOCK) {
      double v = cells_lds[i];
      if (v != 0.0) atomicAdd(&gdst[i], v);
    }
  }
  {
    double* gdst = P.T + P.off.fout;
    for (int i = tid; i < n_esc; i += BLOCK) {
      double v = esc_lds[i];
      if (v != 0.0) atomicAdd(&gdst[i], v);
    }
  }
  flush_counters(P, lc, lane);
}

#if C2D_TABLE_COMTOT
/* Per-step comtot table: tab[cell][g] = sum_i sigma_E(i, x_g) f_nt(cell,i) dg_i
 * (src/comtot2d.f:220-241 without the n_e factor).  sigma_E(i, x_g) does not
 * depend on the cell, so it is evaluated once per run into S[g][i]
 * (c2d_comtab_sigma) and the per-step table is the small GEMM
 * tab = W * S^T with W[cell][i] = f_nt(cell,i) * dg_i. */
__global__ void __launch_bounds__(256) c2d_comtab_sigma(const double* gnt, double* S) {
  const int gi = blockIdx.x;                 /* grid point */
  const double du = (C2D_COMTAB_U1 - C2D_COMTAB_U0) / (double)(C2D_COMTAB_N - 1);
  const double x = c2d_exp(C2D_COMTAB_U0 + du * gi) / EMASSKEV;
  for (int i = threadIdx.x; i < C2D_NUM_NT - 1; i += blockDim.x)
    S[(int64_t)gi * C2D_NUM_NT + i] = sigma_E_bin(gnt[i], x);
  if (threadIdx.x == 0) S[(int64_t)gi * C2D_NUM_NT + C2D_NUM_NT - 1] = 0.0;
}

/* one 64x64 output tile per 256-thread block; K = 200 staged through LDS */
__global__ void __launch_bounds__(256) c2d_comtab_gemm(const double* f_nt, const double* gnt,
                                                       const double* S, double* tab, int ncell) {
  __shared__ double Ws[64][41];
  __shared__ double Ss[64][41];
  const int c0 = blockIdx.y * 64, g0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  double acc[4][4] = {};
  for (int k0 = 0; k0 < C2D_NUM_NT; k0 += 40) {
    for (int e = threadIdx.x; e < 64 * 40; e += 256) {
      const int rr = e / 40, kk = e % 40, k = k0 + kk;
      const int c = c0 + rr, gg = g0 + rr;
      double w = 0.0;
      if (c < ncell && k < C2D_NUM_NT - 1) w = f_nt[(int64_t)c * C2D_NUM_NT + k] * (gnt[k + 1] - gnt[k]);
      Ws[rr][kk] = w;
      Ss[rr][kk] = (gg < C2D_COMTAB_N && k < C2D_NUM_NT) ? S[(int64_t)gg * C2D_NUM_NT + k] : 0.0;
    }
    __syncthreads();
#pragma unroll 4
    for (int kk = 0; kk < 40; kk++) {
      double a[4], b[4];
#pragma unroll
      for (int m = 0; m < 4; m++) a[m] = Ws[ty + 16 * m][kk];
#pragma unroll
      for (int n = 0; n < 4; n++) b[n] = Ss[tx + 16 * n][kk];
#pragma unroll
      for (int m = 0; m < 4; m++)
#pragma unroll
        for (int n = 0; n < 4; n++) acc[m][n] += a[m] * b[n];
    }
    __syncthreads();
  }
#pragma unroll
  for (int m = 0; m < 4; m++)
#pragma unroll
    for (int n = 0; n < 4; n++) {
      const int c = c0 + ty + 16 * m, gg = g0 + tx + 16 * n;
      if (c < ncell && gg < C2D_COMTAB_N) tab[(int64_t)c * C2D_COMTAB_N + gg] = acc[m][n];
    }
}
#endif

}  // namespace c2d

/* ------------------------------------------------------------------ */
/* launchers (called from capi.cpp)                                    */
/* ------------------------------------------------------------------ */
/* trk: c2d_config.trk_variant (0: src/imctrk2d.f, 1: src_20121113) */
extern "C" int C2D_SFX(c2d_launch_transport)(const c2d::KParams* P_dev, const c2d::GenArgs* A, int grid,
                                             size_t lds_bytes, int trk, hipStream_t stream) {
  if (trk)
    hipLaunchKernelGGL(C2D_SFX(c2d::c2d_transport_kernel)<1>, dim3(grid), dim3(c2d::BLOCK), lds_bytes,
                       stream, P_dev, *A);
  else
    hipLaunchKernelGGL(C2D_SFX(c2d::c2d_transport_kernel)<0>, dim3(grid), dim3(c2d::BLOCK), lds_bytes,
                       stream, P_dev, *A);
  return (int)hipGetLastError();
}

static int C2D_SFX(bundle_lds_attr)(size_t lds_bytes) {
  if (lds_bytes <= 64 * 1024) return 0;
  for (const void* k : {(const void*)C2D_SFX(c2d::c2d_bundle_kernel)<0>,
                        (const void*)C2D_SFX(c2d::c2d_bundle_kernel)<1>})
    if (hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes))
      return (int)e;
  return 0;
}

extern "C" int C2D_SFX(c2d_launch_bundle)(const c2d::KParams* P_dev, const c2d::GenArgs* A, int grid,
                                          size_t lds_bytes, int trk, hipStream_t stream) {
  if (int e = C2D_SFX(bundle_lds_attr)(lds_bytes)) return e;
  if (trk)
    hipLaunchKernelGGL(C2D_SFX(c2d::c2d_bundle_kernel)<1>, dim3(grid), dim3(c2d::BLOCK), lds_bytes,
                       stream, P_dev, *A);
  else
    hipLaunchKernelGGL(C2D_SFX(c2d::c2d_bundle_kernel)<0>, dim3(grid), dim3(c2d::BLOCK), lds_bytes,
                       stream, P_dev, *A);
  return (int)hipGetLastError();
}

/* trk: the tracker instance the context launches (c2d_config.trk_variant):
 * its own VGPR count sets the resident blocks */
extern "C" int C2D_SFX(c2d_bundle_occupancy)(int* blocks_per_cu, size_t lds_bytes, int trk) {
  if (C2D_SFX(bundle_lds_attr)(lds_bytes) != 0) { *blocks_per_cu = 0; return 0; }
  return (int)(trk ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                         blocks_per_cu, C2D_SFX(c2d::c2d_bundle_kernel)<1>, c2d::BLOCK, lds_bytes)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                         blocks_per_cu, C2D_SFX(c2d::c2d_bundle_kernel)<0>, c2d::BLOCK, lds_bytes));
}

extern "C" int C2D_SFX(c2d_launch_source)(const c2d::KParams* P_dev, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(C2D_SFX(c2d::c2d_source_kernel), dim3(grid), dim3(c2d::SRCBLOCK), 0, stream, P_dev);
  return (int)hipGetLastError();
}

/* the scatter kernel over items [item_begin, item_end), then the hard list
 * it leaves (A->n_hard zeroed by the caller); hard_grid blocks of SBLOCK */
extern "C" int C2D_SFX(c2d_launch_scatter)(const c2d::KParams* P_dev, const c2d::GenArgs* A, int grid,
                                           int hard_grid, hipStream_t stream) {
  hipLaunchKernelGGL(C2D_SFX(c2d::c2d_scatter_kernel), dim3(grid), dim3(c2d::SBLOCK), 0, stream, P_dev,
                     *A);
  if (hipError_t e = hipGetLastError()) return (int)e;
  hipLaunchKernelGGL(C2D_SFX(c2d::c2d_scatter_hard_kernel), dim3(hard_grid), dim3(c2d::SBLOCK), 0, stream,
                     P_dev, *A);
  return (int)hipGetLastError();
}

/* resident blocks per CU of the source (which = 0) and scatter (1) kernels:
 * their static LDS (Geo image, prefix) limits them below the 8 per CU a
 * plain CUs x 8 grid would assume, leaving a second partial round */
extern "C" int C2D_SFX(c2d_aux_occupancy)(int which, int* blocks_per_cu) {
  hipError_t e = which == 0
      ? hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, C2D_SFX(c2d::c2d_source_kernel), c2d::SRCBLOCK, 0)
      : hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, C2D_SFX(c2d::c2d_scatter_kernel), c2d::SBLOCK, 0);
  return (int)e;
}

extern "C" int C2D_SFX(c2d_transport_occupancy)(int* blocks_per_cu, size_t lds_bytes, int trk) {
  hipError_t e = trk ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                           blocks_per_cu, C2D_SFX(c2d::c2d_transport_kernel)<1>, c2d::BLOCK, lds_bytes)
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                           blocks_per_cu, C2D_SFX(c2d::c2d_transport_kernel)<0>, c2d::BLOCK, lds_bytes);
  return (int)e;
}

#if C2D_TABLE_COMTOT
extern "C" int c2d_launch_comtab_sigma(const double* gnt, double* S, hipStream_t stream) {
  hipLaunchKernelGGL(c2d::c2d_comtab_sigma, dim3(C2D_COMTAB_N), dim3(256), 0, stream, gnt, S);
  return (int)hipGetLastError();
}
extern "C" int c2d_launch_comtab_gemm(const double* f_nt, const double* gnt, const double* S,
                                      double* tab, int ncell, hipStream_t stream) {
  dim3 grid(C2D_COMTAB_N / 64, (ncell + 63) / 64);
  hipLaunchKernelGGL(c2d::c2d_comtab_gemm, grid, dim3(256), 0, stream, f_nt, gnt, S, tab, ncell);
  return (int)hipGetLastError();
}
#endif
