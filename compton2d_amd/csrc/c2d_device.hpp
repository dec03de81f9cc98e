/*
 * c2d_device.hpp — data layout shared by the host C-ABI (capi.cpp) and the
 * transport kernels (transport.hip).
 */
#ifndef C2D_DEVICE_HPP
#define C2D_DEVICE_HPP

#include <stdint.h>
#include "../../include/compton2d.h"

namespace c2d {

/* Run-constant grids, 1-based like the reference COMMON arrays. */
#define C2D_IDX_BUCKETS 2048       /* 128 octaves at 1/16 octave */
struct Geo {
  double z[C2D_MAXZONE + 1];          /* z[0] = zmin, z[1..nz]           */
  double r[C2D_MAXZONE + 1];          /* r[0] = rmin, r[1..nr]           */
  double E_ph[C2D_N_VOL + 1];         /* E_ph[1..400]                    */
  double E_field[C2D_NPHFIELD + 1];   /* E_field[1..400]                 */
  double hu[C2D_NPHOMAX + 2];         /* hu[1..nphtotal+1]               */
  double Elcmin[C2D_NPHLCMAX + 1];
  double Elcmax[C2D_NPHLCMAX + 1];
  double mu[C2D_NMUMAX + 1];
  /* bin lookup without bisection (grid_lookup): the top 16 bits of a
   * positive double (exponent + 4 mantissa bits, 1/16 octave) minus those of
   * the grid's first value select a bucket; *_start[bucket] = the bin of the
   * bucket's smallest double, from which an upward scan of <= 2 bins finds
   * the bin of x.  Built on the host with the bisection's semantics. */
  int16_t eph_start[C2D_IDX_BUCKETS];
  int16_t efl_start[C2D_IDX_BUCKETS];
  int32_t eph_k0, efl_k0;
};
/* LDS image of Geo (everything but nothing else). */
constexpr int GEO_DOUBLES = (int)(sizeof(Geo) / sizeof(double));

struct SpecDev {             /* file_sp table (imcsurf2d_para.f:544-685) */
  int32_t nfile;
  const double* E_file;
  const double* a1;
  const double* I_file;
  const double* F_file;
  const double* P_file;
};

/* Census packet store, SoA (record of imctrk2d.f:558-572 + lineage key). */
/* Census SoA.  Exact build: `phi` is the reference's azimuth.  Fast build
 * (tabulated comtot) stores the azimuth encoded as the flight carries it:
 * `phi` holds Eta = cos(phi) and bit C2D_CENS_ESW of `bins` the quadrant
 * switch (phi > pi or phi < 1e-10), so a census packet costs no acos when it
 * is written and no cos when it is read back; the host decodes and encodes
 * with the same c2d_acos / c2d_cos (c2d_census_export / _import), so the
 * records it sees are the ones the fast kernel wrote before this encoding. */
#define C2D_CENS_ESW (1u << 24)
/* a volume source of this step written in census format by the source
 * kernel (KParams.vol_cens_base): its dcen is c dt U, U the first draw of
 * its own stream (vol_source, imcvol2d_para.f:206), not the census's c dt */
#define C2D_CENS_VOL (1u << 25)
/* Double-buffered census: a wave's unused tail of its last append chunk is
 * marked dead (bins = C2D_CENS_DEAD) and closed by the host's compaction
 * (capi.cpp census_compact). */
#define C2D_CENS_DEAD (1u << 31)
/* Chunked census (census_inplace = 1: one SoA per context, 64 B per record):
 * the SoA is cut into chunks of C2D_CCHUNK slots.  The census is a list of
 * chunks, all full but the last: census item i lives at slot
 * clist[i >> 10] * 1024 + (i & 1023).  A step appends its census writes into
 * wave-private chunks taken from the free pool; the bundle kernel counts the
 * live sources of each census chunk it works on, and a chunk whose sources
 * have all finished goes to the wave's stack of free chunks, taken before
 * the pool; a full stack, and the stack a wave leaves at its end, go to the
 * shared relist, taken after the stack and before the pool (by every wave of
 * the step's launches).  After the step the partly filled chunks (one per wave slot at most)
 * are packed into full ones and the chunks taken become the next list
 * (capi.cpp census_chunks_close). */
#ifndef C2D_CCHUNK_LOG
#define C2D_CCHUNK_LOG 10
#endif
#define C2D_CCHUNK (1 << C2D_CCHUNK_LOG)
#define C2D_CT_TRACK 16      /* census chunks a wave counts down at once (pow 2) */
#define C2D_CT_STACK 8       /* freed chunks a wave holds for its next appends */
/* A census record's jk word: kph | ie << 7 | jph << 16 | efl << 23 (jph, kph
 * <= 99: 7 bits each; ie, efl <= 400: 9 bits each).  ie is the E_ph bin of
 * xnu (the kappa_tot column, imctrk2d.f:382-384) and efl its E_field bin (the
 * n_field row, imctrk2d.f:547-549): xnu does not change between a census
 * write and the next step's read, so a census packet looks neither up
 * again.  Every writer stores both (the kernels, c2d_census_import by the
 * same bisection; c2d_census_append rejects a record with ie = 0): ie is
 * 1..400, efl 1..400 or 0 for xnu at or below the field grid's lower edge
 * (no n_field row, imctrk2d.f:544-549). */
__host__ __device__ __forceinline__ uint32_t c2d_cens_jk(int jph, int kph, int ie, int efl) {
  return (uint32_t)kph | ((uint32_t)ie << 7) | ((uint32_t)jph << 16) | ((uint32_t)efl << 23);
}
__host__ __device__ __forceinline__ int c2d_cens_j(uint32_t jk) { return (int)((jk >> 16) & 0x7fu); }
__host__ __device__ __forceinline__ int c2d_cens_k(uint32_t jk) { return (int)(jk & 0x7fu); }
__host__ __device__ __forceinline__ int c2d_cens_ie(uint32_t jk) { return (int)((jk >> 7) & 0x1ffu); }
__host__ __device__ __forceinline__ int c2d_cens_efl(uint32_t jk) { return (int)(jk >> 23); }

/* The 64-B record as four 16-B columns, so a lane writes and reads a record
 * with four dwordx4 accesses (a wave's access to one column is contiguous):
 *   rz (rpre, zpre), wp (wmu, phi), ex (ew, xnu), tg (jk, bins, key low, key high)
 * jk: c2d_cens_jk (jph, kph 1-based + the E_ph / E_field bins); bins: jgpsp |
 * jgplc << 8 | jgpmu << 16 (| C2D_CENS_ESW | C2D_CENS_VOL | C2D_CENS_DEAD). */
typedef double __attribute__((ext_vector_type(2))) c2d_d2;
typedef uint32_t __attribute__((ext_vector_type(4))) c2d_u4;
struct CensusSoA {
  c2d_d2* rz;
  c2d_d2* wp;
  c2d_d2* ex;
  c2d_u4* tg;
};

/* Collision record: packet state after the move to the collision point
 * (imctrk2d.f:593-604 "csv" copy) plus the RNG point of the split. */
struct ScatRec {
  double rpre, zpre, wmu, phi, ew, xnu, dcen;
  uint32_t jk;
  uint32_t ctr;      /* RNG counter of the parent (SCAT2) / child (SCAT3) */
  uint64_t key;      /* parent key (SCAT2) / child key (SCAT3)            */
  uint32_t kap;      /* 0: census/volume phase kappa (H3), 1: surface phase */
  uint32_t sub;      /* lineage sub-stream of `key` (c2d_rng.h)           */
};

/* In-flight packet store, SoA: generation-0 sources sampled by
 * c2d_source_kernel and scatter secondaries sampled by c2d_scatter_kernel,
 * consumed by the transport kernel (coalesced: lane i reads element i). */
struct PktSoA {
  double* rpre; double* zpre; double* wmu; double* phi; double* ew; double* xnu; double* dcen;
  uint32_t* jk;      /* jph << 16 | kph                                         */
  uint32_t* bins;    /* jgpsp | jgplc << 8 | jgpmu << 16 | kap << 24            */
  uint32_t* ctr;     /* RNG counter position of `key`                           */
  uint32_t* sub;     /* its sub-stream (a split3 copy's successful resample)    */
  uint64_t* key;
};

struct TallyOff {
  int64_t edep, prdep, ecens, npcen, n_field, E_IC, nelectron, fout, edout;
  int64_t erlki, erlko, erlku, erlkl, Ed_in, counters;
};

/* The escape-event buffer is split into C2D_EV_SHARDS equal shards, each
 * with its own append counter (workgroup b appends to shard b % SHARDS), so
 * the per-wave reservations do not all serialise on one address (escapes
 * are the most frequent append: +14 % transport throughput over one shared
 * counter).  Readers take the shards' filled prefixes in shard order. */
#define C2D_EV_SHARDS 32
/* threads per workgroup of the transport/bundle kernels (build-time knob:
 * with C2D_WAVES_PER_EU it sets how many waves per SIMD can be resident) */
#ifndef C2D_TR_BLOCK
#define C2D_TR_BLOCK 256
#endif
#define C2D_EV_SHARD_STRIDE 16
/* generation-0 work items are split into C2D_WORK_SHARDS contiguous ranges,
 * each with its own fetch counter (one per 128-B line); a workgroup starts
 * on shard blockIdx % C2D_WORK_SHARDS and moves on when it is exhausted */
#define C2D_WORK_SHARDS 64

#ifndef C2D_COMTAB_N
#define C2D_COMTAB_N 2048
#endif
/* comtot table: x grid in u = ln(xnu/keV) */
#define C2D_COMTAB_U0 (-27.631021115928547)   /* ln(1e-12) */
#define C2D_COMTAB_U1 (29.933606208922594)    /* ln(1e13)  */

/* fast build (transport.hip TAU_LOG): log(u), u in (0, 1).  Below 1/2:
 * v_log_f32 of (float)u (|log u| > 0.69, so its absolute error is small
 * against it); above: log1p(-v) of the
 * complement v = 1 - u by Kahan's form log(w) * v / (1 - w), w = 1 - v in
 * f32 (a few f32 ulp however small v is) */
__device__ __forceinline__ double c2d_tau_log_f32(double u) {
  const float v = (float)(1.0 - u);
  const float w = 1.0f - v;
  const bool lo = u < 0.5;
  const float lg = 0.69314718f * __builtin_amdgcn_logf(lo ? (float)u : w);
  const float r = (w == 1.0f) ? -v : lg * (v * __builtin_amdgcn_rcpf(1.0f - w));
  return (double)(lo ? lg : r);
}

enum : int32_t {
  ERR_CENSUS = 1, ERR_EVENT = 2, ERR_QUEUE = 4, ERR_SPEC = 8, ERR_NONFINITE = 16
};

/* Explicit global-address-space access for pointers that arrive through
 * KParams (generic pointers): global_load/store/atomic instead of flat ones,
 * which would also count against lgkmcnt and stall LDS waits. */
#define C2D_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ T gld(const T* p) { return *(const C2D_GLOBAL T*)p; }
template <class T>
__device__ __forceinline__ void gst(T* p, T v) { *(C2D_GLOBAL T*)p = v; }
/* census columns (CensusSoA): one 16-B global access each */
__device__ __forceinline__ void cst2(c2d_d2* p, double a, double b) {
  const c2d_d2 v = {a, b};
  *(C2D_GLOBAL c2d_d2*)p = v;
}
__device__ __forceinline__ c2d_d2 cld2(const c2d_d2* p) { return *(const C2D_GLOBAL c2d_d2*)p; }
__device__ __forceinline__ void cst4(c2d_u4* p, uint32_t jk, uint32_t bins, uint64_t key) {
  const c2d_u4 v = {jk, bins, (uint32_t)key, (uint32_t)(key >> 32)};
  *(C2D_GLOBAL c2d_u4*)p = v;
}
__device__ __forceinline__ c2d_u4 cld4(const c2d_u4* p) { return *(const C2D_GLOBAL c2d_u4*)p; }
__device__ __forceinline__ uint64_t c2d_tg_key(c2d_u4 t) { return ((uint64_t)t.w << 32) | (uint64_t)t.z; }
/* the same accesses marked non-temporal (read or written once per step:
 * the census stream through the transport kernels, C2D_CENS_NT) */
__device__ __forceinline__ void cst2_nt(c2d_d2* p, double a, double b) {
  const c2d_d2 v = {a, b};
  __builtin_nontemporal_store(v, (C2D_GLOBAL c2d_d2*)p);
}
__device__ __forceinline__ c2d_d2 cld2_nt(const c2d_d2* p) {
  return __builtin_nontemporal_load((const C2D_GLOBAL c2d_d2*)p);
}
__device__ __forceinline__ void cst4_nt(c2d_u4* p, uint32_t jk, uint32_t bins, uint64_t key) {
  const c2d_u4 v = {jk, bins, (uint32_t)key, (uint32_t)(key >> 32)};
  __builtin_nontemporal_store(v, (C2D_GLOBAL c2d_u4*)p);
}
__device__ __forceinline__ c2d_u4 cld4_nt(const c2d_u4* p) {
  return __builtin_nontemporal_load((const C2D_GLOBAL c2d_u4*)p);
}
/* a record's bins word alone (compaction scans, dead marks) */
__device__ __forceinline__ uint32_t cens_bins(const c2d_u4* tg, int64_t s) {
  return gld(reinterpret_cast<const uint32_t*>(tg + s) + 1);
}
__device__ __forceinline__ void cens_set_bins(c2d_u4* tg, int64_t s, uint32_t b) {
  gst(reinterpret_cast<uint32_t*>(tg + s) + 1, b);
}
__device__ __forceinline__ void gadd(double* p, double v) {
  __hip_atomic_fetch_add((C2D_GLOBAL double*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void gor(int32_t* p, int32_t v) {
  __hip_atomic_fetch_or((C2D_GLOBAL int32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* n_field census tallies go to C2D_NF_REPL replicas (workgroup b adds to
 * replica b mod C2D_NF_REPL), summed into the tally buffer after the last
 * generation.  f64 atomics execute at the memory side and serialise per
 * address; packets that census together share (cell, energy bin), so a single
 * copy is a hot spot (2.5x on the EC light-curve workload).  8 replicas (one
 * per XCD under the usual round-robin placement, a speed matter only) beat 16
 * and 32 on C3 generation 0 (124.2/124.0 vs 124.6/124.7 vs 125.1/125.2 ms)
 * with C5 unchanged (profiles/r05q); 128 lost 2 % (r05n). */
#ifndef C2D_NF_REPL
#define C2D_NF_REPL 8
#endif

/* internal counter slot (not part of the tally buffer's counters, zeroed
 * before the counters are copied there): lane path-steps = passes of a lane
 * through the geometry block.  The per-copy tracker counts one per
 * packet-step; the bundle kernel one per shared step of all copies on the
 * path.  The roofline's algorithmic bytes are priced on it. */
#define C2D_CNT_PATHS_INT 10
/* internal counter slots: census slots marked dead (double-buffered census:
 * the unused tails of the append chunks); chunked census: chunks recycled
 * within the step, and census chunks whose sources the bundle kernel could
 * not count down (all C2D_CT_TRACK slots busy, or the free stack full) */
#define C2D_CNT_DEAD_INT 12
#define C2D_CNT_CREUSE_INT 13
#define C2D_CNT_CLOST_INT 14

struct KParams {
  int32_t nz, nr, ncell, nphtotal, nph_lc, nmu;
  int32_t split1, split2, split3, spl3_trg, spec_switch;
  int32_t rank, world, ncycle, eps_linear;
  double time, dt, rmin, zmin, cdt;
  double cens_wlim;         /* census records' |wmu| clamp: 0.99999999 (src), 1 (trk_variant 2012-11) */
  uint64_t step_key;
  const Geo* geo;
  const double* gnt;        /* [200] */
  const double* kappa_cv;   /* [ncell][400] census + volume phase (H3) */
  const double* kappa_s;    /* [ncell][400] surface phase               */
  const double* eps_tot;    /* [ncell][400] */
  const double* eps_th;
  const double* f_nt;       /* [ncell][200] */
  const double* Pnt;
  const double* n_e;        /* [ncell] */
  const double* vfrac;      /* [ncell][4] f_thermal, f_inn, f_outer, f_upper */
  const double* ewsv;       /* [ncell] */
  const int64_t* vol_prefix;    /* [ncell+1] global volume-source prefix */
  const int64_t* surf_prefix;   /* [nslot+1] global surface-source prefix */
  const double* surf_ew;        /* [nslot] */
  const double* surf_tbb;       /* [nslot] */
  const int32_t* surf_spec;     /* [nslot] */
  const double* tbbl;           /* [nr]  lower-surface temperature (imcleak) */
  const SpecDev* spectra;
  int32_t n_spectra, nslot;
  const double* comtab;         /* [ncell][C2D_COMTAB_N] cosig on the u grid, f64 (as the
                                   reference evaluates comtot; 16 KB per cell)               */
  double comtab_du_inv;
  double egg_min;            /* E_field(1)^2 / E_field(2): n_field threshold (imctrk2d.f:547-556) */
  /* census: double-buffered cin -> cout (clist null), or one chunked SoA
   * (cin == cout, clist = the input's chunk list); cap_cout = physical slots */
  CensusSoA cin, cout;
  int64_t n_cin, cap_cout;
  uint32_t cens_chunk;       /* census slots per wave reservation */
  unsigned long long* n_cout;
  const int32_t* clist;      /* chunked: census item i at clist[i >> 10] * 1024 + (i & 1023) */
  const int32_t* pool;       /* chunked: free chunks at the step's start ...            */
  const unsigned long long* pool_n;   /* ... how many                                    */
  unsigned long long* pool_head;      /* ... taken so far                                */
  int32_t* out_list;         /* chunked: every chunk the step took, in order of taking   */
  unsigned long long* n_out;
  int32_t* relist;           /* chunked: freed chunks waves handed on (-1: not yet written) */
  unsigned long long* n_relist;
  unsigned long long* relist_head;
  int64_t* cstate;           /* [2 * wave slot]: its partly filled chunk (first slot or -1,
                                used) from launch to launch; closed after the step      */
  /* events */
  double* ev;
  int64_t cap_ev;
  unsigned long long* n_ev_sh;   /* [C2D_EV_SHARDS * C2D_EV_SHARD_STRIDE] shard counters */
  int64_t cap_ev_sh;             /* events per shard                                    */
  /* scatter queues */
  int64_t cap_q;
  /* packet store (sources of generation 0 / secondaries of generation >= 1) */
  PktSoA pk;
  int64_t cap_pk;
  /* this step's work */
  int64_t n_cens_items, n_vol_items, n_surf_items;
  /* >= 0: the source kernel writes the volume sources in census format into
   * cin at slots [vol_cens_base, + n_vol_items) and generation 0 takes them
   * as census items (prefetched like them); -1: the packet store */
  int64_t vol_cens_base;
  int64_t n_vol_global, n_surf_global;
  /* tallies */
  double* T;
  double* nf_rep;           /* C2D_NF_REPL replicas of n_field, [r][cell][nphfield] */
  TallyOff off;
  unsigned long long* cnt;  /* [C2D_NCOUNTERS] */
  int32_t* err;
  int32_t lds_cells;        /* 1: cell tallies privatised in LDS */
  unsigned long long* prof;  /* [C2D_TR_PROF_WORDS] section counters (-DC2D_TR_PROF builds) */
  /* guide rows of the emission CDFs (eps_linear == 0): cdf_guide[(t * ncell + cell) *
   * (C2D_CDF_GUIDE + 1) + q] = the smallest i in [1, 400] with cdf(i) >= q / C2D_CDF_GUIDE
   * (400 if none), t 0: eps_tot, 1: eps_th; null: the full binary search */
  const uint16_t* cdf_guide;
};
#define C2D_CDF_GUIDE 256

/* Per-launch arguments (passed by value; KParams stays constant over a step). */
/* scatter kernels' defaults (GenArgs.kn_cap, GenArgs.sc_k1; transport.hip) */
#define C2D_KN_CAP_DEFAULT 32
#define C2D_SC_K1_DEFAULT 16
struct GenArgs {
  const ScatRec* q2_in;            /* scatter kernel: this generation's records   */
  const ScatRec* q3_in;
  ScatRec* q2_out;                 /* transport kernel: collisions -> next gen    */
  ScatRec* q3_out;                 /* scatter kernel: third splits -> next gen    */
  unsigned long long* n2_out;
  unsigned long long* n3_out;
  unsigned long long* n_pk;        /* scatter: secondaries written; transport: item count */
  unsigned long long* work_counter;
  unsigned long long* work_sh;     /* bundle kernel: C2D_WORK_SHARDS counters, stride 16 */
  unsigned long long* n_hard;      /* scatter: split3 copies left for the hard kernel */
  int64_t* hard;                   /* their item indices (capacity KParams.cap_pk)  */
  int64_t item_begin, item_end;    /* scatter kernel item range                   */
  int64_t n_items;                 /* transport, generation 0: census + sources    */
  int64_t n2_in, n3_in;
  int32_t gen;
  int32_t kn_cap;                  /* scatter: compb2d first-loop iterations a lane runs alone
                                      before the wave resolves it (C2D_KN_CAP_ITERS test knob) */
  int32_t sc_k1;                   /* scatter: split3 attempts per lane before the hard list
                                      (C2D_SC_K1_ATTEMPTS test knob) */
};

/* ---- emission / absorption tables (vem.hip) ---- */
/* per-cell input record [ncell][VZ_N], packed by the host */
enum : int32_t {
  VZ_TEA = 0, VZ_TNA, VZ_NE, VZ_B, VZ_FPAIR, VZ_ZSURF, VZ_VOL, VZ_EP, VZ_LMIN, VZ_N = 12
};
/* per-cell output record [ncell][VO_N] */
enum : int32_t { VO_B = 0, VO_ESY, VO_ECY, VO_ETH, VO_ETOT, VO_N = 8 };
struct VemParams {
  const double* zin;      /* [ncell][VZ_N]          */
  const double* f_nt;     /* [ncell][NUM_NT]        */
  const double* gnt;      /* [NUM_NT]               */
  const double* E_ph;     /* [N_VOL] photon grid    */
  const double* mcd;      /* McDonald abscissae (C2D_FP_MCD_N x 4) */
  double dE, pow3_15, dt; /* grid ratio, 3**1.5, dt(1) */
  double* kappa;          /* [ncell][N_VOL] outputs */
  double* eps_tot;
  double* eps_th;
  double* zout;           /* [ncell][VO_N]          */
};

/* ---- Fokker-Planck solve (fp.hip) ---- */
/* per-zone input record [ncell][FZ_N], packed by the host */
enum : int32_t {
  FZ_VOL = 0, FZ_TEA, FZ_TNA, FZ_NE, FZ_B, FZ_ELSY, FZ_ECENS, FZ_ECOLD, FZ_TURB, FZ_FPAIR,
  FZ_PNTH, FZ_N = 16
};
/* per-zone output record [ncell][FO_N]: state, then C2D_FP_NDIAG diagnostics */
enum : int32_t { FO_TE = 0, FO_NE, FO_GMIN, FO_GMAX, FO_AMXWL, FO_PNTH, FO_DIAG = 8, FO_N = 16 };
enum : int32_t { FPERR_STEPS = 1, FPERR_GUARD = 2, FPERR_NF_IN = 4, FPERR_NF_OUT = 8 };

/* McDonald abscissa table: n < C2D_FP_MCD_N -> {t_n, ts_n, (ts_n^2-1)^1.5, (ts_n^2-1)^2.5} */
#define C2D_FP_MCD_N 16384
/* the fast kernel's McDonald moment table (fp_fast.hip, C2D_FPF_MTAB): z0 on
 * a geometric grid of C2D_FPF_MT_Q points per octave from 2^C2D_FPF_MT_LO to
 * 2^C2D_FPF_MT_HI; per entry C2D_FPF_MT_W doubles: z0, 1/z0, the two series'
 * stopping indices f at z0, C2D_FPF_MT_K moments of each series, and each
 * series' abscissa rows (t, ts, p) at n = f-1 .. f+2 */
#define C2D_FPF_MT_Q 1024
#define C2D_FPF_MT_LO (-17)
#define C2D_FPF_MT_HI 3
#define C2D_FPF_MT_N ((C2D_FPF_MT_HI - C2D_FPF_MT_LO) * C2D_FPF_MT_Q + 1)
#define C2D_FPF_MT_K 7
#define C2D_FPF_MT_W (4 + 2 * C2D_FPF_MT_K + 24)

struct FpParams {
  int32_t nz, nr, pick_sw, inj_switch, inj_dis, g2var_switch, cf_sentinel, pair_sw;
  double time, dt, df_implicit, df_T, r_esc, r_acc;
  double r_flare, z_flare, t_flare, sigma_r, sigma_z, sigma_t, flare_amp;
  double inj_g1, inj_g2, inj_p, inj_t, inj_L, pick_rate, inj_gg, inj_sigma, inj_v;
  const Geo* geo;          /* grids: z[0]=zmin, r[0]=rmin, 1-based zones      */
  const double* gnt;       /* [num_nt]                                         */
  const double* FT;        /* [nphfield][num_nt]: F_IC transposed               */
  const double* mcd;       /* [C2D_FP_MCD_N][4] McDonald table                 */
  const double* zin;       /* [ncell][FZ_N]                                    */
  const double* f_in;      /* [ncell][num_nt]                                  */
  const double* P_in;      /* [ncell][num_nt]                                  */
  const double* nf;        /* n_field: nf[cell*nphfield + ph]                  */
  const double* ecens;     /* [ncell] (tally buffer) or null: zin[FZ_ECENS]     */
  double* f_out;           /* [ncell][num_nt]                                  */
  double* P_out;
  double* zout;            /* [ncell][FO_N]                                    */
  int32_t* err;
  /* gamma_bar memo shared by every zone and step (fp.hip GbMemo): keys are
   * the bits of Theta (0 = empty), values gamma_bar (0 = not yet written) */
  unsigned long long* gb_key;
  double* gb_val;
  uint32_t gb_mask;        /* slots - 1 (power of two)                         */
  /* fast kernel only: zones taken from a queue, zorder[q] the q-th zone
   * (costliest first, from the previous update's sub-step counts) */
  const int32_t* zorder;   /* [ncell] or null: q-th zone = q                  */
  int32_t* zq;             /* queue head, zeroed before the launch            */
  int32_t ncell;
  /* fast kernel: the McDonald moment table (null: every pair by its series),
   * and whether the shared gamma_bar memo is still consulted beside it */
  const double* mom;       /* [C2D_FPF_MT_N][C2D_FPF_MT_W]                    */
  int32_t mt_glob;
  /* fast kernel: 1 = cost probe, every zone stops after its first implicit
   * sub-step's f_t_implicit and writes 1/f_t_implicit to its sub-step count */
  int32_t probe;
};

/* ---- observer-frame binning (observe.hip) ---- */
struct ObsDev {
  double gam_bulk, rmax, t_offset;
  int32_t mode, n_t, n_mu, n_e;
  const double* t0; const double* t1;
  const double* mu0; const double* mu1;
  const double* E0; const double* E1;
  double* F;                 /* [n_t][n_mu][n_e] sum of ew       */
  double* F2;                /* sum of ew^2                        */
  double* cnt;               /* particle counts (exact integers)  */
  int32_t lds_rows;          /* leading time rows privatised in LDS (0..n_t) */
  int32_t sorted_t, sorted_mu, sorted_e;   /* lo[] and hi[] non-decreasing: binary search */
};

}  // namespace c2d

#endif
