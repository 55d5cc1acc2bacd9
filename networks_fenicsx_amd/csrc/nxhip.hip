// nxhip.hip -- MI355X (gfx950) assemble + MINRES path for the hydraulic network
// saddle-point system of networks_fenicsx. C ABI in include/nxhip.h.
//
// Reference semantics (files under /root/reference/src/networks_fenicsx/):
//   forms            assembly.py:243-277 (mass, divergence, gradient, junctions, rhs)
//   assemble         assembly.py:328-368, solver.py:90-101
//   solve            solver.py:107-135 (PETSc KSP; MUMPS LU by default) -> MINRES here
//   mesh geometry    mesh.py:269-322 (interior points x_u (1-w) + x_v w, w = k/N)
//
// Layout per rank (see include/nxhip.h): edge e owns rows [e(2N+1), (e+1)(2N+1)),
// interleaved q_0 p_0 q_1 ... p_{N-1} q_N, then the owned multipliers. With this
// order an edge's CSR rows form ONE contiguous segment of 7N+1(+1 per junction end)
// entries, so the assembly kernel writes every value with unit-stride stores and
// the SpMV gathers x from a +-2 band (plus the far multiplier columns).
//
// Pressure rows are negated (and their rhs) so A is symmetric; MINRES needs that.

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../include/nxhip.h"

#define NX_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kVersion = 1 * 10000 + 1 * 100 + 0;  // 1.1: nx_create_fe, nx_set_source
constexpr int kBlock = 256;         // threads per block (4 wave64)
constexpr int kRowsPerBlock = 256;  // SpMV: one row per thread
constexpr int kLdsCap = 2048;       // SpMV: products staged per block (16 KiB)
constexpr int kReduceThreads = 1024;

thread_local std::string g_err;

// Phase timing (debug builds only, -DNX_PHASE_TIMING: scripts/phase_timing.py). Workgroup 0
// stamps wall_clock64() (100 MHz) at phase boundaries; every workgroup raises the latest
// start / end of its kernel. Slot bases: k_mr_a 0, up 16, top 32, down 48, coarse 64.
#ifdef NX_PHASE_TIMING
__device__ unsigned long long g_phase[128];
__device__ unsigned long long g_wgs[8][512];  // per-workgroup start / end, last launch wins
__device__ unsigned long long g_wge[8][512];
__device__ unsigned long long g_dst[48][512];  // k_dir_step: per-workgroup stamps (nx_debug_dstep)
#define NX_DSTAMP(k)                                                   \
  do {                                                                 \
    if (threadIdx.x == 0 && blockIdx.x < 512) g_dst[(k)][blockIdx.x] = wall_clock64(); \
  } while (0)
// store-site ledger of the one-launch step (scripts/store_ledger.py, NXHIP_LEDGER): a set bit
// drops one class of its global stores (1 CSR values, 2 rhs, 4 x, 16 multiplier rows'
// values) so that WRITE_SIZE differences attribute the written bytes -- debug build only
#define NX_LEDGER(da, bit) (((da).ledger & (bit)) != 0)
#define NX_PHASE(slot)                                           \
  do {                                                           \
    if (blockIdx.x == 0) {                                       \
      __syncthreads();                                           \
      if (threadIdx.x == 0) g_phase[(slot)] = wall_clock64();    \
    }                                                            \
  } while (0)
#define NX_PHASE_START(base)                                                        \
  do {                                                                              \
    if (threadIdx.x == 0) {                                                         \
      const unsigned long long t_ = wall_clock64();                                 \
      if (blockIdx.x == 0) g_phase[(base)] = t_;                                    \
      atomicMax(&g_phase[(base) + 14], t_);                                         \
      if (blockIdx.x < 512) g_wgs[(base) / 16][blockIdx.x] = t_;                    \
    }                                                                               \
  } while (0)
#define NX_PHASE_END(base)                                                          \
  do {                                                                              \
    __syncthreads();                                                                \
    if (threadIdx.x == 0) {                                                         \
      const unsigned long long t_ = wall_clock64();                                 \
      atomicMax(&g_phase[(base) + 15], t_);                                         \
      if (blockIdx.x < 512) g_wge[(base) / 16][blockIdx.x] = t_;                    \
    }                                                                               \
  } while (0)
#else
#define NX_PHASE(slot) \
  do {                 \
  } while (0)
#define NX_PHASE_START(base) \
  do {                       \
  } while (0)
#define NX_PHASE_END(base) \
  do {                     \
  } while (0)
#define NX_DSTAMP(k) \
  do {               \
  } while (0)
#define NX_LEDGER(da, bit) false
#endif

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCALL(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(NX_ERR_HIP, std::string(#expr) + " failed: " + hipGetErrorString(e_)); \
  } while (0)

#define NCCLCALL(expr)                                                                      \
  do {                                                                                      \
    ncclResult_t r_ = (expr);                                                               \
    if (r_ != ncclSuccess)                                                                  \
      return fail(NX_ERR_RCCL, std::string(#expr) + " failed: " + ncclGetErrorString(r_)); \
  } while (0)

#define CHECK(expr)      \
  do {                   \
    int rc_ = (expr);    \
    if (rc_ != NX_OK) return rc_; \
  } while (0)

// ------------------------------------------------------------------------------------
// Entry decoding of one edge's CSR segment. With s = (source is a bifurcation), the
// segment is   [q_0: 3+s][p_0: 2][q_1: 5][p_1: 2] ... [q_{N-1}: 5][p_{N-1}: 2][q_N: 3+t]
// Columns are edge-local DoFs (2k = q_k, 2k+1 = p_k) or LM_SRC / LM_DST.
enum : int { V_P1 = 0, V_M1 = 1, V_MD = 2, V_MO = 3, V_MD2 = 4 };
constexpr int LM_SRC = -1, LM_DST = -2;

struct Entry {
  int row, col, vk, cell;
};

__device__ __forceinline__ Entry decode_entry(int i, int N, int s) {
  Entry en;
  const int q0len = 3 + s;
  if (i < q0len) {  // row q_0: [q_0, p_0, q_1, (lambda_src)]
    en.row = 0;
    en.cell = 0;
    en.col = (i < 3) ? i : LM_SRC;
    en.vk = (i == 0) ? V_MD : (i == 1) ? V_P1 : (i == 2) ? V_MO : V_M1;
    return en;
  }
  const int i1 = i - q0len;
  const int g = i1 / 7;
  const int r = i1 - 7 * g;
  if (g < N - 1) {
    if (r < 2) {  // row p_g (negated divergence): +1 at q_g, -1 at q_{g+1}
      en.row = 2 * g + 1;
      en.col = 2 * g + 2 * r;
      en.vk = r ? V_M1 : V_P1;
      en.cell = g;
    } else {  // interior row q_{g+1}: [q_g, p_g, q_{g+1}, p_{g+1}, q_{g+2}]
      const int j = r - 2;
      en.row = 2 * g + 2;
      en.col = 2 * g + j;
      en.vk = (j == 0) ? V_MO : (j == 1) ? V_M1 : (j == 2) ? V_MD2 : (j == 3) ? V_P1 : V_MO;
      en.cell = (j == 4) ? g + 1 : g;
    }
    return en;
  }
  const int i2 = i1 - 7 * (N - 1);
  if (i2 < 2) {  // row p_{N-1}
    en.row = 2 * N - 1;
    en.col = 2 * (N - 1) + 2 * i2;
    en.vk = i2 ? V_M1 : V_P1;
    en.cell = N - 1;
    return en;
  }
  const int j = i2 - 2;  // row q_N: [q_{N-1}, p_{N-1}, q_N, (lambda_dst)]
  en.row = 2 * N;
  en.cell = N - 1;
  en.col = (j < 3) ? 2 * N - 2 + j : LM_DST;
  en.vk = (j == 0) ? V_MO : (j == 1) ? V_M1 : (j == 2) ? V_MD : V_P1;
  return en;
}

// Start of row q_k inside the segment (k = 0..N), and segment length.
__device__ __forceinline__ int q_row_start(int k, int s) { return k == 0 ? 0 : s + 7 * k - 2; }

struct EdgeArgs {
  const double* edge_x;  // E*6
  const int* edge_lm;    // E*2
  const int* edge_seg;   // E+1 segment offsets into the CSR arrays
  int64_t E;
  int N;
};

// ------------------------------------------------------------------------------------
// Pattern: one wave per edge writes the row pointers of its 2N+1 rows and the column
// indices of its segment (unit stride across lanes).
__global__ __launch_bounds__(kBlock) void k_pattern(EdgeArgs ea, int* __restrict__ rowptr,
                                                      int* __restrict__ colidx) {
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (e >= ea.E) return;
  const int N = ea.N;
  const int lm0 = ea.edge_lm[2 * e], lm1 = ea.edge_lm[2 * e + 1];
  const int s = lm0 >= 0;
  const int seg = ea.edge_seg[e];
  const int len = ea.edge_seg[e + 1] - seg;
  const int64_t base = e * (2 * N + 1);
  for (int i = lane; i < len; i += 64) {
    const Entry en = decode_entry(i, N, s);
    const int gcol = en.col >= 0 ? (int)(base + en.col) : (en.col == LM_SRC ? lm0 : lm1);
    colidx[seg + i] = gcol;
    if (i == 0 || decode_entry(i - 1, N, s).row != en.row) rowptr[base + en.row] = seg + i;
  }
}

// ------------------------------------------------------------------------------------
// Assembly: one wave per edge. Cells are processed in chunks of 64 (lane = cell):
// each lane regenerates its cell's vertices exactly like the reference mesh
// generator and computes the P1 mass element tensor (R h/3, R h/6); then the wave
// writes the chunk's CSR values (unit stride), fetching neighbouring cells' tensors by
// cross-lane permutes (no LDS, no barriers). A register carries the previous chunk's
// last cell.
struct AsmArgs {
  EdgeArgs ea;
  const double* edge_R;   // E (per-edge R)
  const double* edge_bc;  // E*2 rhs at q_0 / q_N
  double f;
  const double* edge_f;   // E per-edge source, or nullptr: f everywhere
  double* val;
  double* rhs;
  double* dq;  // E*(N+1) lumped flux mass (preconditioner), or nullptr
  int lhs, do_rhs;
  // multiplier rows: +-1 values and zero rhs, done by the blocks after the edge blocks
  int edge_blocks;
  int64_t nnz_lm, B;
  const double* lm_val;
  double* val_lm;
  double* rhs_lm;
};

__device__ __forceinline__ void vertex(const double* x0, const double* x1, int k, int N,
                                       double invN, double* p) {
#pragma clang fp contract(off)
  if (k == 0) {
    p[0] = x0[0]; p[1] = x0[1]; p[2] = x0[2];
  } else if (k == N) {
    p[0] = x1[0]; p[1] = x1[1]; p[2] = x1[2];
  } else {
    // numpy: w = k * (1/N); start * (1 - w) + end * w   (mesh.py:275, 290)
    const double w = (double)k * invN;
    const double om = 1.0 - w;
    p[0] = x0[0] * om + x1[0] * w;
    p[1] = x0[1] * om + x1[1] * w;
    p[2] = x0[2] * om + x1[2] * w;
  }
}

// Small N (N < S <= 32): 64 / S edges per wave, one S-lane segment per edge (lane = cell).
// The wave's edges own one contiguous CSR range, written unit-stride by all 64 lanes;
// entry -> edge by the (at most 4) segment boundaries. Same arithmetic as k_assemble.
template <int S>
__global__ __launch_bounds__(kBlock) void k_assemble_seg(AsmArgs a) {
#pragma clang fp contract(off)
  constexpr int EPW = 64 / S;
  if ((int)blockIdx.x >= a.edge_blocks) {  // multiplier rows: +-1 values, zero rhs
    const int64_t i = (int64_t)(blockIdx.x - a.edge_blocks) * kBlock + threadIdx.x;
    if (a.lhs && i < a.nnz_lm) a.val_lm[i] = a.lm_val[i];
    if (a.do_rhs && i < a.B) a.rhs_lm[i] = 0.0;
    return;
  }
  const int lane = threadIdx.x & 63;
  const int sub = lane / S, cl = lane % S;
  const int64_t e0 = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * EPW;
  if (e0 >= a.ea.E) return;  // wave-uniform
  const int64_t E = a.ea.E;
  const int ne = (int)min<int64_t>(EPW, E - e0);
  const int64_t e = e0 + min(sub, ne - 1);  // idle segments shadow the last edge
  const bool mine = sub < ne;
  const int N = a.ea.N;
  const double invN = 1.0 / (double)N;
  double x0[3], x1[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    x0[c] = a.ea.edge_x[6 * e + c];
    x1[c] = a.ea.edge_x[6 * e + 3 + c];
  }
  const double R = a.edge_R[e];
  const int s = a.ea.edge_lm[2 * e] >= 0;
  const int seg = a.ea.edge_seg[e];
  const int64_t base = e * (2 * N + 1);
  double md = 0.0, mo = 0.0;
  if (mine && cl < N) {
    double pa[3], pb[3];
    vertex(x0, x1, cl, N, invN, pa);
    vertex(x0, x1, cl + 1, N, invN, pb);
    const double d0 = pb[0] - pa[0], d1 = pb[1] - pa[1], d2 = pb[2] - pa[2];
    const double h = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
    md = R * h / 3.0;
    mo = R * h / 6.0;
    if (a.do_rhs) {
      const double fe = a.edge_f ? a.edge_f[e] : a.f;
      a.rhs[base + 2 * cl + 1] = -(fe * h);  // negated pressure row: -(f h)
      a.rhs[base + 2 * cl] = (cl == 0) ? a.edge_bc[2 * e] : 0.0;
    }
  }
  if (mine && a.do_rhs && cl == N) a.rhs[base + 2 * N] = a.edge_bc[2 * e + 1];
  // neighbours' tensors: cell cl - 1 (the lumped mass) and the last cell (q_N)
  const int sb = sub * S;
  const double mdL = __shfl(md, sb + max(cl - 1, 0), 64), moL = __shfl(mo, sb + max(cl - 1, 0), 64);
  // lumped flux mass (the preconditioner's D block): with the values or on its own (the
  // direct solve's graph writes rhs + dq first and the values on a second branch)
  if (a.dq != nullptr && mine && cl <= N) {
    double d;
    if (cl < N) {
      d = md + mo;
      if (cl > 0) d = (moL + mdL) + d;
    } else {
      d = moL + mdL;  // q_N: the last cell only
    }
    a.dq[e * (int64_t)(N + 1) + cl] = d;
  }
  if (a.lhs) {
    // the wave's contiguous CSR range [b_0, b_ne)
    int bnd[EPW + 1], sfl[EPW];
#pragma unroll
    for (int j = 0; j < EPW; ++j) {
      bnd[j] = __shfl(seg, j * S, 64);
      sfl[j] = __shfl(s, j * S, 64);
    }
    const int last = a.ea.edge_seg[e0 + ne];
    bnd[EPW] = last;
#pragma unroll
    for (int j = 0; j < EPW; ++j)
      if (j >= ne) bnd[j] = last;
    for (int ib = bnd[0]; ib < last; ib += 64) {  // uniform trip count across the wave
      const int i = ib + lane;
      int j = 0;
#pragma unroll
      for (int t = 1; t < EPW; ++t) j += (i >= bnd[t]) ? 1 : 0;
      int sj = sfl[0], b0 = bnd[0];
#pragma unroll
      for (int t = 1; t < EPW; ++t)
        if (t == j) {
          sj = sfl[t];
          b0 = bnd[t];
        }
      const Entry en = decode_entry(i < last ? i - b0 : 0, N, sj);
      const int src = j * S + en.cell;
      const double mdA = __shfl(md, src, 64), moA = __shfl(mo, src, 64);
      const double mdB = __shfl(md, min(src + 1, 63), 64);
      double v;
      switch (en.vk) {
        case V_P1: v = 1.0; break;
        case V_M1: v = -1.0; break;
        case V_MD: v = mdA; break;
        case V_MO: v = moA; break;
        default: v = mdA + mdB; break;  // interior diagonal: cells g and g+1
      }
      if (i < last) a.val[i] = v;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_assemble(AsmArgs a) {
#pragma clang fp contract(off)
  if ((int)blockIdx.x >= a.edge_blocks) {  // multiplier rows: +-1 values, zero rhs
    // (assembly.py:271-277; L[lm] = 0)
    const int64_t i = (int64_t)(blockIdx.x - a.edge_blocks) * kBlock + threadIdx.x;
    if (a.lhs && i < a.nnz_lm) a.val_lm[i] = a.lm_val[i];
    if (a.do_rhs && i < a.B) a.rhs_lm[i] = 0.0;
    return;
  }
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (e >= a.ea.E) return;  // wave-uniform; the waves of a block never synchronise
  const int N = a.ea.N;
  const double invN = 1.0 / (double)N;
  double x0[3], x1[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    x0[c] = a.ea.edge_x[6 * e + c];
    x1[c] = a.ea.edge_x[6 * e + 3 + c];
  }
  const double R = a.edge_R[e];
  const int s = a.ea.edge_lm[2 * e] >= 0;
  const int seg = a.ea.edge_seg[e];
  const int seglen = a.ea.edge_seg[e + 1] - seg;
  const int64_t base = e * (2 * N + 1);
  const double bc0 = a.edge_bc[2 * e], bc1 = a.edge_bc[2 * e + 1];
  const double fe_src = a.edge_f ? a.edge_f[e] : a.f;
  // the previous chunk's last cell (slot 0 of the chunk)
  double md_prev = 0.0, mo_prev = 0.0;
  for (int c0 = 0; c0 < N; c0 += 64) {
    const int nc = min(64, N - c0);
    double md = 0.0, mo = 0.0;  // this lane's cell c0 + lane: R h/3, R h/6
    if (lane < nc) {
      const int k = c0 + lane;
      double pa[3], pb[3];
      vertex(x0, x1, k, N, invN, pa);
      vertex(x0, x1, k + 1, N, invN, pb);
      const double d0 = pb[0] - pa[0], d1 = pb[1] - pa[1], d2 = pb[2] - pa[2];
      const double h = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
      md = R * h / 3.0;
      mo = R * h / 6.0;
      if (a.do_rhs) {
        a.rhs[base + 2 * k + 1] = -(fe_src * h);  // negated pressure row: -(f h)
        a.rhs[base + 2 * k] = (k == 0) ? bc0 : 0.0;
      }
    }
    if (a.do_rhs && lane == 0 && c0 + nc == N) a.rhs[base + 2 * N] = bc1;
    if (a.lhs) {
      // the chunk's CSR entries, unit stride; element tensors of neighbouring lanes come
      // by cross-lane permutes (slot = cell - c0 + 1, slot 0 = previous chunk's last cell)
      const int i0 = q_row_start(c0, s);
      const int i1 = (c0 + nc == N) ? seglen : q_row_start(c0 + nc, s);
      for (int ib = i0; ib < i1; ib += 64) {  // uniform trip count across the wave
        const int i = ib + lane;
        const Entry en = decode_entry(i < i1 ? i : i0, N, s);
        const int slot = en.cell - c0 + 1;  // in [0, nc]
        const double mdA = __shfl(md, max(slot - 1, 0), 64);
        const double moA = __shfl(mo, max(slot - 1, 0), 64);
        const double mdB = __shfl(md, min(slot, 63), 64);
        const double md_s = slot == 0 ? md_prev : mdA, mo_s = slot == 0 ? mo_prev : moA;
        double v;
        switch (en.vk) {
          case V_P1: v = 1.0; break;
          case V_M1: v = -1.0; break;
          case V_MD: v = md_s; break;
          case V_MO: v = mo_s; break;
          default: v = md_s + mdB; break;  // interior diagonal: cells g and g+1
        }
        if (i < i1) a.val[seg + i] = v;
      }
    }
    // lumped (row-sum) flux mass of q_k, k in the chunk (and q_N in the last chunk):
    // the preconditioner's D block (with the values or on its own, see k_assemble_seg)
    const double mdL = __shfl(md, max(lane - 1, 0), 64), moL = __shfl(mo, max(lane - 1, 0), 64);
    const double mdLast = __shfl(md, nc - 1, 64), moLast = __shfl(mo, nc - 1, 64);
    if (a.dq != nullptr) {
      const int64_t qb = e * (int64_t)(N + 1);
      if (lane < nc) {
        const int k = c0 + lane;
        double d = md + mo;
        if (k > 0) d = (lane > 0 ? moL + mdL : mo_prev + md_prev) + d;
        a.dq[qb + k] = d;
      }
      if (lane == 0 && c0 + nc == N) a.dq[qb + N] = moLast + mdLast;
    }
    md_prev = mdLast;
    mo_prev = moLast;
  }
}


// ------------------------------------------------------------------------------------
// Reductions: deterministic (fixed grid, fixed order), no atomics.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Hand-offs between the workgroups of ONE launch (k_dir_step): write-through stores and
// loads of agent scope (global_store / global_load ... sc1; MI355X_MICROARCH.md,
// inter-workgroup visibility, "stores all sc1 / loads all sc1" with one agent-scope atomic
// per storing workgroup after every storing wave's vmcnt(0)). No release fence, so the
// XCD's L2 -- dirty with CSR values and x -- is not written back on the critical path.
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
  return __builtin_bit_cast(
      double, __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<double*>(p)),
                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
template <bool WT>
__device__ __forceinline__ double ldv(const double* p) {
  if constexpr (WT) return ld_wt(p);
  return *p;
}
template <bool WT>
__device__ __forceinline__ void stv(double* p, double v) {
  if constexpr (WT) st_wt(p, v);
  else *p = v;
}
// every wave's outstanding vector-memory operations (its write-through stores) complete
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// One wave's LDS writes visible to its own later LDS reads (other lanes): the LDS serves a
// wave's requests in order; this keeps the compiler from moving them across (no workgroup
// barrier: the other waves may be elsewhere)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Block of kBlock threads -> one partial per block.
__device__ __forceinline__ void block_sum_store(double v, double* out) {
  __shared__ double s_w[kBlock / 64];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = s_w[0];
#pragma unroll
    for (int i = 1; i < kBlock / 64; ++i) t += s_w[i];
    *out = t;
  }
}

// Sum n partials with one kReduceThreads block; result valid in thread 0.
__device__ __forceinline__ double reduce_partials(const double* __restrict__ p, int n) {
  __shared__ double s_w[kReduceThreads / 64];
  double v = 0.0;
  for (int i = threadIdx.x; i < n; i += kReduceThreads) v += p[i];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0) {
    t = s_w[0];
    for (int i = 1; i < kReduceThreads / 64; ++i) t += s_w[i];
  }
  return t;
}

__global__ __launch_bounds__(kReduceThreads) void k_reduce(const double* __restrict__ p, int n,
                                                          double* __restrict__ out) {
  const double t = reduce_partials(p, n);
  if (threadIdx.x == 0) *out = t;
}

// ------------------------------------------------------------------------------------
// CSR SpMV, "stream" form: the block's nonzeros (contiguous because its rows are)
// are multiplied with the gathered x in one unit-stride sweep and staged in LDS;
// then each thread sums its own row. Sum order is left-to-right per row in both
// branches (no FMA), so results do not depend on the branch taken.
struct Csr {
  const int* rowptr;
  const int* col;
  const double* val;
  int64_t n_rows;
};

__device__ __forceinline__ double spmv_row_sum(const Csr& A, const double* __restrict__ x,
                                               int64_t r0, int nr) {
#pragma clang fp contract(off)
  __shared__ int s_rp[kRowsPerBlock + 1];
  __shared__ double s_prod[kLdsCap];
  const int tid = threadIdx.x;
  for (int i = tid; i <= nr; i += kBlock) s_rp[i] = A.rowptr[r0 + i];
  __syncthreads();
  const int k0 = s_rp[0], k1 = s_rp[nr];
  double sum = 0.0;
  if (k1 - k0 <= kLdsCap) {
    for (int k = k0 + tid; k < k1; k += kBlock) s_prod[k - k0] = A.val[k] * x[A.col[k]];
    __syncthreads();
    if (tid < nr) {
      const int a = s_rp[tid] - k0, b = s_rp[tid + 1] - k0;
      for (int k = a; k < b; ++k) sum += s_prod[k];
    }
  } else if (tid < nr) {
    for (int k = s_rp[tid]; k < s_rp[tid + 1]; ++k) {
      const double p = A.val[k] * x[A.col[k]];
      sum += p;
    }
  }
  return sum;
}

__global__ __launch_bounds__(kBlock) void k_spmv(Csr A, const double* __restrict__ x,
                                                 double* __restrict__ y) {
  const int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlock;
  const int nr = (int)min<int64_t>(kRowsPerBlock, A.n_rows - r0);
  const double s = spmv_row_sum(A, x, r0, nr);
  if ((int)threadIdx.x < nr) y[r0 + threadIdx.x] = s;
}

// residual r = b - A x, partial ||r||^2 and ||b||^2; r itself into rout when given
__global__ __launch_bounds__(kBlock) void k_residual(Csr A, const double* __restrict__ x,
                                                     const double* __restrict__ b,
                                                     double* __restrict__ partials, int nblk,
                                                     double* __restrict__ rout) {
  const int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlock;
  const int nr = (int)min<int64_t>(kRowsPerBlock, A.n_rows - r0);
  const double s = spmv_row_sum(A, x, r0, nr);
  double rr = 0.0, bb = 0.0;
  if ((int)threadIdx.x < nr) {
    const double bv = b[r0 + threadIdx.x];
    const double rv = bv - s;
    if (rout) rout[r0 + threadIdx.x] = rv;
    rr = rv * rv;
    bb = bv * bv;
  }
  block_sum_store(rr, partials + blockIdx.x);
  __syncthreads();
  block_sum_store(bb, partials + nblk + blockIdx.x);
}

// The direct solve's check: the same residual, `ck` 256-row chunks per block (fewer partials
// for the publish step to sum). Swept on MI355X (r02g, profiles/r02g_sweep.log): C3 (1 M rows)
// 1: 0.0883-0.0896, 2: 0.0855-0.0876, 4: 0.089 ms/step; C4 (10 M rows) 1: 1.136, 4: 1.105.
int res_chunks(int64_t n) { return n > (int64_t(4) << 20) ? 4 : 2; }
__global__ __launch_bounds__(kBlock) void k_residual_ck(Csr A, const double* __restrict__ x,
                                                        const double* __restrict__ b,
                                                        double* __restrict__ partials, int nblk,
                                                        double* __restrict__ rout, int ck) {
  double rr = 0.0, bb = 0.0;
  for (int c = 0; c < ck; ++c) {
    const int64_t r0 = ((int64_t)blockIdx.x * ck + c) * kRowsPerBlock;
    if (r0 >= A.n_rows) break;  // block-uniform
    const int nr = (int)min<int64_t>(kRowsPerBlock, A.n_rows - r0);
    const double s = spmv_row_sum(A, x, r0, nr);
    if ((int)threadIdx.x < nr) {
      const double bv = b[r0 + threadIdx.x];
      const double rv = bv - s;
      if (rout) rout[r0 + threadIdx.x] = rv;
      rr += rv * rv;
      bb += bv * bv;
    }
    __syncthreads();  // spmv_row_sum's LDS is reused by the next chunk
  }
  block_sum_store(rr, partials + blockIdx.x);
  __syncthreads();
  block_sum_store(bb, partials + nblk + blockIdx.x);
}

// ------------------------------------------------------------------------------------
// MINRES: Paige & Saunders (1975) recurrences in the form of scipy.sparse.linalg.minres
// (unpreconditioned, shift 0). One iteration k (1-based) = 2 launches on one GPU:
//   k_mr_a(k)  every block, redundantly: beta_k^2 = sum of k_mr_b(k-1)'s partials ->
//              Givens rotation of iteration k-1 -> its pending solution update
//              (w, x), fused with y = A v_k - beta_k v_{k-1} (v_k = r2/beta_k, gathered)
//              and the block partial of alpha_k = v_k . y. Block 0 persists the state.
//   k_mr_b(k)  every block, redundantly: alpha_k = sum of k_mr_a(k)'s partials;
//              r2' = y - (alpha_k / beta_k) r2 and the block partial of ||r2'||^2.
// No atomics and no reduction launches: each kernel re-reduces the previous launch's
// few partials (nA ~ n/1024, nB = 512; L2-resident) in a fixed order, so every block
// computes bit-identical scalars. The state is double-buffered -- k_mr_a(k) reads
// S[(k+1)&1] and writes S[k&1] -- so block 0 can write while other blocks still read.
// The kernel that detects convergence applies the last solution update and stops;
// every later launch of the chunk returns at once.
// Several ranks: partial sums go through k_reduce_slot + an RCCL all-reduce of one
// double (red[0] = alpha, red[1] = beta^2, red[2] = ||b||^2) and the kernels read it.
// r1/r2 swap roles every iteration and w1/w2 too; the host passes the pointers.
constexpr int kChunksADefault = 2;   // k_mr_a: chunks of 256 rows per block (swept: 1,2,4)
constexpr int kBlocksBDefault = 512;  // k_mr_b / start: grid-stride vector kernels

struct MrState {
  double beta1, beta, oldb, alfa, dbar, epsln, phibar, cs, sn, tnorm2, relres, rtol;
  int nb;  // completed Lanczos steps (k_mr_b launches that ran)
  int it;  // completed MINRES iterations (rotations applied)
  int maxit, done, converged, pad;
};

struct Rot {
  double oldeps, delta, denom, phi;
};

// Rotation of iteration it+1 from b2 = beta_{it+2}^2 (scipy minres.py statement order).
__device__ __forceinline__ Rot mr_rotate(MrState& s, double b2) {
  const double alfa = s.alfa, oldb = s.beta, beta = sqrt(b2);
  s.oldb = oldb;
  s.beta = beta;
  s.tnorm2 += alfa * alfa + oldb * oldb + beta * beta;
  Rot r;
  r.oldeps = s.epsln;
  r.delta = s.cs * s.dbar + s.sn * alfa;
  const double gbar = s.sn * s.dbar - s.cs * alfa;
  s.epsln = s.sn * beta;
  s.dbar = -s.cs * beta;
  const double gamma = fmax(hypot(gbar, beta), 2.220446049250313e-16);
  s.cs = gbar / gamma;
  s.sn = beta / gamma;
  r.phi = s.cs * s.phibar;
  s.phibar = s.sn * s.phibar;
  r.denom = 1.0 / gamma;
  s.it += 1;
  s.relres = s.phibar / s.beta1;
  if (s.relres <= s.rtol || beta == 0.0) {
    s.done = 1;
    s.converged = 1;
  } else if (s.it >= s.maxit || !(s.relres == s.relres)) {
    s.done = 1;
  }
  return r;
}

// Sum of n values in a fixed order, identical in every block; returned to all threads.
template <int BS = kBlock>
__device__ __forceinline__ double block_partial(const double* __restrict__ p, int n) {
  double v = 0.0;  // this thread's share, in the fixed order every block uses
  for (int i = threadIdx.x; i < n; i += BS) v += p[i];
  return v;
}

template <int BS = kBlock>
__device__ __forceinline__ double block_allsum_v(double v) {
  __shared__ double s_w[BS / 64];
  __shared__ double s_tot;
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = s_w[0];
#pragma unroll
    for (int i = 1; i < BS / 64; ++i) t += s_w[i];
    s_tot = t;
  }
  __syncthreads();
  return s_tot;
}

template <int BS = kBlock>
__device__ __forceinline__ double block_allsum(const double* __restrict__ p, int n) {
  return block_allsum_v<BS>(block_partial<BS>(p, n));
}

// Block sum of one value per thread -> *out (thread 0). Block size BS.
template <int BS>
__device__ __forceinline__ void block_sum_store_n(double v, double* out) {
  __shared__ double s_w[BS / 64];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = s_w[0];
#pragma unroll
    for (int i = 1; i < BS / 64; ++i) t += s_w[i];
    *out = t;
  }
}

struct MrVecs {
  double* r1;        // out: y
  const double* r1in;  // in: r_{k-1} (usually r1; the rhs at k = 2 of the head graph)
  const double* r2;  // r_k; without preconditioner r_k = beta_k v_k and it is gathered
  double* w1;        // w_{k-3} in, w_{k-1} out (in place)
  const double* w2;  // w_{k-2}
  double* x;
  const double* z;   // preconditioned: z_k = P^{-1} r_k, gathered (has ghost slots)
  double* v;         // preconditioned: v_{k-1} in, v_k = z_k / beta_k out (in place)
  // preconditioned, stored Lanczos vectors (or null): v_1..v_kMaxV live in vs (stride
  // vstride); the first kMaxV rotations only record (oldeps, delta, 1/gamma, phi) in hist
  // and the solution is formed once, x = sum c_i v_i, when the solve stops -- or, past
  // kMaxV iterations, x, w_{m-1}, w_m are formed and the w recurrence takes over
  double* vs;
  int64_t vstride;
  double* hist;
};
constexpr int kMaxV = 8;

// Initial state from beta_1^2 (k_mr_init, or k_mr_a of iteration 1 in the single-rank head
// graph, which folds the initialisation in).
__device__ __forceinline__ MrState mr_initial(double bb, double rtol, int maxit) {
  const double beta1 = sqrt(bb);
  MrState s{};
  s.beta1 = beta1;
  s.beta = beta1;
  s.phibar = beta1;
  s.cs = -1.0;
  s.rtol = rtol;
  s.maxit = maxit;
  s.relres = beta1 > 0.0 ? 1.0 : 0.0;
  if (beta1 == 0.0) {
    s.done = 1;
    s.converged = 1;
  }
  return s;
}

struct MrInit {  // on = 1: iteration 1 starts the solve from beta_1^2 = sum(part[0..np))
  int on;
  int np;
  int maxit;
  double rtol;
  const double* part;
  // lean path: the last k_mr_a of a graph publishes the state it ends with to a host-
  // coherent mapped mirror, stamped with a sequence number (pad) the host waits for --
  // the host learns the outcome without a stream synchronisation or a copy
  int mark;
  int* seq;         // device counter of published states
  MrState* mirror;
};

__device__ __forceinline__ void mr_publish(MrState s, const MrInit& ini) {
  const int q = *ini.seq + 1;
  *ini.seq = q;
  s.pad = 0;
  *ini.mirror = s;
  __threadfence_system();
  __hip_atomic_store(&ini.mirror->pad, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// w_{k-3}, w_{k-2} and x are not initialised in memory: the first rotations read them as
// zero (it0 = completed rotations before this one), so the solve needs no memsets.
template <bool MULTI, bool PC>
__global__ __launch_bounds__(kBlock, 8) void k_mr_a(Csr A, MrVecs v, const MrState* __restrict__ sin,
                                                 MrState* __restrict__ sout,
                                                 const double* __restrict__ partB, int nB,
                                                 const double* __restrict__ red,
                                                 double* __restrict__ partA, int chunksA,
                                                 MrInit ini) {
  // the partials of beta^2 are loaded with the state, not after it (one round trip less)
  const double pB = MULTI || ini.on ? 0.0 : block_partial(partB, nB);
  if (!ini.on && sin->done) {
    if (ini.mark && blockIdx.x == 0 && threadIdx.x == 0) mr_publish(*sin, ini);
    return;
  }
  NX_PHASE_START(0);
  MrState s = ini.on ? mr_initial(block_allsum(ini.part, ini.np), ini.rtol, ini.maxit) : *sin;
  Rot rot{0.0, 0.0, 0.0, 0.0};
  const bool upd = s.nb > 0;  // a Lanczos step is waiting for its rotation
  const int it0 = s.it;
  if (upd) rot = mr_rotate(s, MULTI ? red[1] : block_allsum_v(pB));
  NX_PHASE(1);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *sout = s;
    if (ini.on) *const_cast<MrState*>(sin) = s;  // both buffers start identical
    if (ini.mark) mr_publish(s, ini);
  }
  if (ini.on && s.done) return;  // b = 0
  const double beta = s.beta, oldb = s.oldb;  // beta_k, beta_{k-1}
  const double sc = 1.0 / beta;
  const double c1 = upd ? beta / oldb : 0.0;
  const bool spmv = !s.done;
  const double* g = PC ? v.z : v.r2;  // v_k = g / beta_k
  // stored Lanczos vectors: rotation j = s.it uses v_j = vs[j - 1]
  const bool sv = PC && v.vs != nullptr;
  const int jr = s.it;
  const bool stored = sv && upd && jr <= kMaxV;
  const bool trans = stored && !s.done && jr == kMaxV;  // hand over to the w recurrence
  const bool comb = stored && (s.done || trans);        // form x (and w) from v_1..v_j
  __shared__ double sM[kMaxV][kMaxV], sCx[kMaxV], sH[kMaxV][4];
  if (stored && blockIdx.x == 0 && threadIdx.x == 0) {
    double* hst = v.hist + 4 * (jr - 1);
    hst[0] = rot.oldeps;
    hst[1] = rot.delta;
    hst[2] = rot.denom;
    hst[3] = rot.phi;
  }
  if (comb) {  // w_i = sum_c M[i][c] v_c (the recurrence in coefficients), x = sum phi_i w_i
    // (LDS work arrays: a private 8x8 array would cost every launch its registers)
    const int t = threadIdx.x;
    if (t < 4 * kMaxV) {
      const int i = t >> 2, f = t & 3;
      if (i + 1 < jr) sH[i][f] = v.hist[t];
      else if (i + 1 == jr) sH[i][f] = f == 0 ? rot.oldeps : f == 1 ? rot.delta : f == 2 ? rot.denom : rot.phi;
    }
    __syncthreads();
    if (t < kMaxV) {  // column t of M, rows in order
      double cx = 0.0, m2 = 0.0, m1 = 0.0;
      for (int i = 0; i < jr; ++i) {
        const double m = ((t == i ? 1.0 : 0.0) - sH[i][0] * m2 - sH[i][1] * m1) * sH[i][2];
        sM[i][t] = m;
        cx += sH[i][3] * m;
        m2 = m1;
        m1 = m;
      }
      sCx[t] = cx;
    }
    __syncthreads();
  }
  double* vout = (sv && s.nb < kMaxV) ? v.vs + (int64_t)s.nb * v.vstride : v.v;
  double part = 0.0;
  for (int c = 0; c < chunksA; ++c) {
    const int64_t r0 = ((int64_t)blockIdx.x * chunksA + c) * kRowsPerBlock;
    if (r0 >= A.n_rows) break;
    const int nr = (int)min<int64_t>(kRowsPerBlock, A.n_rows - r0);
    const double Ay = spmv ? spmv_row_sum(A, g, r0, nr) : 0.0;
    if ((int)threadIdx.x < nr) {
      const int64_t r = r0 + threadIdx.x;
      // c1 = 0 in iteration 1; after the last rotation only the solution update remains
      const double r1v = (upd && (spmv || !PC)) ? v.r1in[r] : 0.0;
      if (comb) {  // x (and, handing over, w_{j-1} -> w2's buffer, w_j -> w1's) from v_1..v_j
        double xs = 0.0, wa = 0.0, wb = 0.0;
        // four stored vectors per round, their loads issued together (same summation order)
#pragma unroll 1
        for (int i0 = 0; i0 < jr; i0 += 4) {
          double vi[4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
            vi[u] = i0 + u < jr ? v.vs[(int64_t)(i0 + u) * v.vstride + r] : 0.0;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int i = i0 + u;
            if (i >= jr) break;
            xs += sCx[i] * vi[u];
            if (trans) {
              wa += sM[jr - 2][i] * vi[u];  // w_{j-1}
              wb += sM[jr - 1][i] * vi[u];  // w_j
            }
          }
        }
        v.x[r] = xs;
        if (trans) {
          const_cast<double*>(v.w2)[r] = wa;
          v.w1[r] = wb;
        }
      } else if (upd && !stored) {  // w = (v - oldeps w1 - delta w2) / gamma ; x += phi w
        const double vk = PC ? v.v[r] : r1v / oldb;
        const double w1v = it0 >= 2 ? v.w1[r] : 0.0;  // w_{k-3}, w_{k-2}: zero at first
        const double w2v = it0 >= 1 ? v.w2[r] : 0.0;
        const double wn = (vk - rot.oldeps * w1v - rot.delta * w2v) * rot.denom;
        if (spmv) v.w1[r] = wn;  // no later rotation reads it once the solve stopped
        v.x[r] = (it0 >= 1 ? v.x[r] : 0.0) + rot.phi * wn;
      }
      if (spmv) {
        const double vn = sc * g[r];
        const double y = sc * Ay - c1 * r1v;
        part += vn * y;
        v.r1[r] = y;
        if (PC) vout[r] = vn;
      }
    }
    __syncthreads();  // LDS of spmv_row_sum is reused by the next chunk
  }
  NX_PHASE(2);
  if (spmv) block_sum_store(part, partA + blockIdx.x);
  NX_PHASE_END(0);
}

template <bool MULTI>
__global__ __launch_bounds__(kBlock) void k_mr_b(int64_t n, double* __restrict__ y,
                                                 const double* __restrict__ r2,
                                                 MrState* __restrict__ st,
                                                 MrState* __restrict__ other,
                                                 const double* __restrict__ partA, int nA,
                                                 const double* __restrict__ red,
                                                 double* __restrict__ partB) {
  if (st->done) {
    // k_mr_a of this iteration stopped the solve: make the other buffer final too, or
    // the k_mr_a two launches later would resume from its stale (not done) copy
    if (blockIdx.x == 0 && threadIdx.x == 0) *other = *st;
    return;
  }
  const double beta = st->beta;
  const double alfa = MULTI ? red[0] : block_allsum(partA, nA);
  const double c2 = alfa / beta;
  double part = 0.0;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const double v = y[i] - c2 * r2[i];
    y[i] = v;
    part += v * v;
  }
  block_sum_store(part, partB + blockIdx.x);
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // fields no other block reads here
    st->alfa = alfa;
    st->nb += 1;
  }
}

// ||b||^2 partials for the start
__global__ __launch_bounds__(kBlock) void k_sumsq(const double* __restrict__ b, int64_t n,
                                                  double* __restrict__ part) {
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    acc += b[i] * b[i];
  block_sum_store(acc, part + blockIdx.x);
}

template <bool MULTI>
__global__ __launch_bounds__(kBlock) void k_mr_init(const double* __restrict__ part, int np,
                                                    const double* __restrict__ red,
                                                    MrState* __restrict__ st, double rtol,
                                                    int maxit) {
  const double bb = MULTI ? red[2] : block_allsum(part, np);
  if (threadIdx.x == 0) *st = mr_initial(bb, rtol, maxit);
}

// Reduce partials into red[slot] (multi-rank: then all-reduced).
__global__ __launch_bounds__(kBlock) void k_reduce_slot(const double* __restrict__ part, int n,
                                                        double* __restrict__ red, int slot) {
  const double t = block_allsum(part, n);
  if (threadIdx.x == 0) red[slot] = t;
}

// ------------------------------------------------------------------------------------
// Tree Schur-complement preconditioner z = P^{-1} r, P = blockdiag(D, G^T D^{-1} G)
// (networks_fenicsx_amd/precond.py has the derivation and the host decomposition).
// Per iteration: k_pc_up (lower subtrees + chain-only jobs: Lanczos update of r, chain
// condensation, junction elimination inside each subtree) -> k_pc_top (one workgroup:
// junctions above the cut, solve, back-substitution) -> k_pc_down (subtree back-
// substitution, chain cells by the 1-D Green's function, z and partial r.z).
// A chain is processed by a W-lane segment, CPL cells per lane (N <= W*CPL).
struct PcArgs {
  int N;
  // 1 / N, formed once on the host (correctly rounded: the device's 1.0 / (double)N, bit for
  // bit) -- a uniform the fused kernels would otherwise form in VGPRs and spill
  double invN;
  const int* chain_edge;
  const int* chain_flip;
  const int* chain_up;
  const int* chain_lo;
  const int* slot_lam;
  const int* slot_pchain;
  const int* slot_parent;
  const int* slot_dc_off;
  const int* slot_dc;
  const int* dc_lo;      // bottom slot of every slot_dc entry (host-precomputed)
  const int* slot_plam;  // multiplier row of the parent slot, -1
  const int* job_chain_off;
  const int* job_lvl_off;
  const int* lvl_slot_off;
  const int* top_lvl_off;
  int n_top_lvl;
  int n_jobs;
  const double* dq;  // E*(N+1) lumped flux mass
  double* chain_T;
  double* chain_It;
  double* chain_Ib;
  double* slot_D;
  double* slot_J;
  double* slot_A;  // back-substitution z_j = A_j + B_j z_parent (LDS kernels)
  double* slot_B;
  // coarse step (several ranks, precond.py): coarse index of every slot, local chains
  // joining two coarse junctions (top / bottom coarse index; the bottom one is the child
  // and indexes the conductance), the global coarse forest, and the exchange buffer
  // [D | J | G] (3 n_coarse doubles) that is all-reduced between the two halves
  int n_coarse;
  int n_cc;
  int n_clvl;
  const int* slot_cidx;
  const int* cc_chain;
  const int* cc_top;
  const int* cc_bot;
  const int* c_parent;
  const int* c_child_off;
  const int* c_child;
  const int* c_lvl_off;
  // per coarse junction k its coarse chains in chain order (ck_off: n_coarse + 1; ck_ent:
  // i << 1 | (k is the chain's bottom)): pc_coarse_partials' sums without scanning them all
  const int* ck_off;
  const int* ck_ent;
  double* cbuf;
  // linear form (several ranks, LDS kernels): the sweeps condense y instead of
  // r' = y - (alpha/beta) r2 and the down sweep forms z = P^{-1}y - (alpha/beta) z_old,
  // so alpha's partial rides in the coarse all-reduce (xalpha = cbuf + 3 n_coarse)
  int lin;
  const double* xalpha;
  // dense inverse of the coarse forest system (n_coarse^2, built per solve by k_pc_gc in
  // the start application; null when n_coarse > kCapCoarseLds): the fused down sweeps form
  // z_c = Gc J_c by dot products instead of the level sweeps
  double* Gc;
  double* slot_z;  // P^{-1}y at every junction slot (written by the top part, read across jobs)
  // dense top part (single rank, LDS kernels; precond.py: _dense_top_lists): G = inverse
  // of the top tree Schur matrix (n_top^2, built once per solve by k_pc_gbuild); per job
  // the top slots it updates / writes and the top slots whose values it needs
  int dense;
  int n_top;
  const int* job_tslot_off;
  const int* job_tslot;
  const int* job_need_off;
  const int* job_need;
  double* G;
  // producer-side top inputs: a_s = sum u[top_uoff[s] .. top_uoff[s+1])
  const int* top_uoff;
  const int* slot_uy;
  const int* chain_uit;
  const int* chain_uib;
  const int* job_root_u;
  const int* job_root_dc;
  double* u;
  // factored coefficients (single rank, once per solve by k_pc_factor; D is fixed by the
  // assembly): kappa = g / D_child per hanging-chain entry (0 when grounded), 1 / D
  int factored;
  double* dc_kappa;
  double* slot_invD;
  // dense top with several ranks (mdense): the top trees are rooted at coarse junctions
  // (Dirichlet): z_t = G[t,:] a + w_t zc[root(t)], and the coarse partial J of a root r is
  // KJ[r,:] a; atop = a (k_pc_cpart), zc = the coarse solution (k_pc_coarse)
  int mdense;
  double* KJ;
  double* top_w;
  int* top_rootc;
  double* atop;
  double* zc;
  // exact Schur complement (default): P = blockdiag(M, G^T M^{-1} G) with the consistent
  // flux mass M instead of its lumped D (precond.py: "Exact variant"). The junction system
  // is the same; only the chain outputs change: z_q = M_e^{-1} r_q (M_e = mo T per edge,
  // mo = R h / 6, T = tridiag(1, 4, 1), 2 at both ends, solved by Thomas scans with the
  // host-computed pivots Tlu = [l_k | 1/u_k]) and z_p = z_p(lumped) - mo r_p.
  // MINRES then converges in 3 iterations (3 distinct eigenvalues of P^{-1} A).
  int exact;
  const double* Tlu;
  int n_dc_all, n_slots_all;  // hanging-chain entries / junction slots (k_pc_factor sizes)
  // several ranks, dense top, LDS kernels, small coarse forest (nx_set_coarse): the up
  // sweep's last workgroup does k_pc_cpart's work (ticket[0]) and every down workgroup
  // solves the coarse forest itself, so neither one-workgroup kernel runs per iteration;
  // fuse_pack (one-graph solve): the down sweep's last workgroup (ticket[1]) also packs the
  // halo and this rank's beta^2 (k_pack_beta's work)
  int fused;
  int fuse_pack;
  // direct solve, refinement pass: the sweeps add their output to x instead of storing it
  int accum;
  int* ticket;
  const int* send_idx;
  int n_send;
  double* send_buf;
  double* red1;
  double* gath_self;
  // direct solve, one rank: the true residual r = b - A x is formed by the down sweep from
  // the values it just computed (direct_residual): its chains' rows and the multiplier rows
  // of the junctions whose chains are all in its job (slot_rloc); k_dir_publish_fr does the
  // rest from the CSR. edge_x / edge_R regenerate the cell masses exactly as k_assemble does.
  int fres;
  const double* edge_x;
  const double* edge_R;
  const int* slot_rloc;
  const double* rhs_b;  // the assembled rhs b (a refinement pass checks b - A (x + d))
  double* rres;   // r (kept for a refinement step)
  double* rpart;  // per job: partial ||r||^2, then (n_jobs on) partial ||b||^2
  int top_reg;    // k_pc_top_lds: register level sweeps allowed
  // the up sweep's one-wave junction levels, set up by the host: per job kmax + 1 (0: the
  // job runs the block-wide levels), per lower slot [level | nk << 8, child 0 | child 1 << 16,
  // child 2 | child 3 << 16] with child = local slot | dc offset << 6
  const int* job_wave;
  const int* slot_wave;
  // the top part's register level sweeps, host-built (top_body): per top slot its level and
  // junction-children count (lv | nk << 8), then kWaveKids entries child | (dc offset << 12);
  // null when a slot has more children or the top part exceeds one workgroup
  const int* top_wave;
  // the flux mass of one cell is R h [[a, b], [b, a]] (P1: a = 1/3, b = 1/6; a (k, 0) system
  // condensed to its vertex fluxes: element.condensed_flux_mass): mo = b R h of a chain is
  // its end flux's lumped mass (a + b) R h / mo_div, mo_div = (a + b) / b (P1: 3)
  double mo_div;
  int topdown;    // one rank, direct: the top part solved in every down sweep workgroup
  int coarsedown;  // several ranks, direct: the coarse step (k_pc_coarse) in every one
  // small coarse forests (<= 64 junctions, <= kWaveKids children): per junction
  // [level | nk << 8 | (parent + 1) << 12, children packed 8 bits each] (nx_set_coarse), so
  // the one-wave coarse solve needs no staging (coarse_wave_solve)
  const int* c_wave;
  // the top part as wave subtrees (round 4, host-built; null: the level sweeps of top_wave):
  // every maximal subtree of <= 64 slots is swept by one wave with shuffles (lane = slot, no
  // barriers), the few slots above them ("upper", top_sub_nup levels) by the level sweeps.
  // top_sub: per top slot (1 + kWaveKids) ints as top_wave for upper slots (word 0 with bit
  // 31 set), word 0 = 0 for subtree members; top_lane: per thread of the top part's
  // workgroup [slot or -1, lane | depth << 6 | nk << 14 | parent lane << 18, kWaveKids x
  // (child lane | dc offset << 12)]; top_sub_dep: per wave its subtree's depth (0: none)
  const int* top_sub;
  const int* top_lane;
  const int* top_sub_dep;
  int top_sub_nup;
  int top_ts0, top_nt, top_dc0, top_ndc;  // the top part's slots and hanging-chain entries
};

constexpr int kCapCoarseLds = 256;  // coarse forests the down workgroups solve in LDS

// This rank's share of the coarse system: the eliminated (D, J) of its coarse slots (all
// in the top part, level 0) and the chains joining two coarse junctions. sD/sJ are indexed
// by top-part position. Ends with the buffer complete (one workgroup). WT: the chains' data
// were handed over inside the launch (k_dir_team_up): write-through loads.
template <int BS, bool WT = false>
__device__ __forceinline__ void pc_coarse_partials(const PcArgs& pa, int ts0, int nt, const double* sD,
                                   const double* sJ) {
  // small coarse sets: the buffer is built in LDS and the coarse chains' data loaded in
  // parallel (thread = chain), then every coarse junction sums its chains in chain order
  // (thread = junction; the additions of one thread walking the chains) and writes out
  // (was: built in global memory, two dependent round trips plus a read-modify-write per
  // chain on thread 0 -- ~14 us on the ranks holding the tree's upper part, 8-rank rehearsal)
  constexpr int kCapCC = 256;
  __shared__ double sBuf[3 * kCapCC], sCg[kCapCC], sCit[kCapCC], sCib[kCapCC];
  __shared__ int sCt[kCapCC], sCb[kCapCC];
  const int nC = pa.n_coarse, ncc = pa.n_cc;
  const bool lds = nC <= kCapCC && ncc <= kCapCC;
  double* __restrict__ buf = lds ? sBuf : pa.cbuf;
  for (int i = threadIdx.x; i < 3 * nC; i += BS) buf[i] = 0.0;
  __syncthreads();
  for (int sl = threadIdx.x; sl < nt; sl += BS) {
    const int k = pa.slot_cidx[ts0 + sl];
    if (k >= 0) {
      buf[k] = sD[sl];
      buf[nC + k] = sJ[sl];
    }
  }
  if (lds)
    for (int i = threadIdx.x; i < ncc; i += BS) {
      const int c = pa.cc_chain[i];
      sCt[i] = pa.cc_top[i];
      sCb[i] = pa.cc_bot[i];
      sCg[i] = 1.0 / ldv<WT>(pa.chain_T + c);
      sCit[i] = ldv<WT>(pa.chain_It + c);
      sCib[i] = ldv<WT>(pa.chain_Ib + c);
    }
  __syncthreads();
  if (lds) {  // thread = coarse junction k: its sums over the chains in chain order (the same
              // additions in the same order as one thread walking the chains)
    for (int k = threadIdx.x; k < nC; k += BS) {
      double D = sBuf[k], J = sBuf[nC + k], Gk = sBuf[2 * nC + k];
      if (pa.ck_off) {  // its own chains only (host-listed in chain order)
        for (int e = pa.ck_off[k]; e < pa.ck_off[k + 1]; ++e) {
          const int en = pa.ck_ent[e], i = en >> 1;
          D += sCg[i];
          if (en & 1) {
            J += sCib[i];
            Gk = sCg[i];
          } else {
            J += sCit[i];
          }
        }
      } else {
        for (int i = 0; i < ncc; ++i) {
          const int t = sCt[i], b = sCb[i];
          if (t == k) {
            D += sCg[i];
            J += sCit[i];
          }
          if (b == k) {
            D += sCg[i];
            J += sCib[i];
            Gk = sCg[i];
          }
        }
      }
      pa.cbuf[k] = D;
      pa.cbuf[nC + k] = J;
      pa.cbuf[2 * nC + k] = Gk;
    }
    return;
  }
  if (threadIdx.x == 0) {  // large coarse sets: one thread, in global memory, same order
    for (int i = 0; i < ncc; ++i) {
      const int c = pa.cc_chain[i];
      const int t = pa.cc_top[i], b = pa.cc_bot[i];
      const double g = 1.0 / ldv<WT>(pa.chain_T + c);
      buf[t] += g;
      buf[b] += g;
      buf[nC + t] += ldv<WT>(pa.chain_It + c);
      buf[nC + b] += ldv<WT>(pa.chain_Ib + c);
      buf[2 * nC + b] = g;
    }
  }
}

// The lane's position in its chain, formed afresh where a helper needs it: the values
// derived from it (cell indices) then live only inside the helper instead of through phase 2
// (k_dir_step spilled two of them to scratch at its 128-VGPR budget)
template <int W>
__device__ __forceinline__ int lane_of() {
  int l = threadIdx.x & (W - 1);
  asm volatile("" : "+v"(l));
  return l;
}

template <int W>
__device__ __forceinline__ double seg_incl_scan(double v) {
  const int l = threadIdx.x & (W - 1);
#pragma unroll
  for (int o = 1; o < W; o <<= 1) {
    const double t = __shfl_up(v, o, W);
    if (l >= o) v += t;
  }
  return v;
}

template <int W>
__device__ __forceinline__ double seg_sum(double v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, W);
  return v;
}

// Cells / fluxes of one chain seen by one lane: chain order runs top -> bottom.
template <int W, int CPL>
struct ChainLane {
  int valid[CPL];
  int dof_c[CPL];  // pressure DoF of chain cell k = l*CPL + t (rows are int32, as in the CSR)
  int dof_q[CPL];  // flux DoF of chain q_k (between cell k-1 and k)
  double rho[CPL];
  double D[CPL];       // resistance distance top -> cell k
  int has_last;        // this lane also owns q_N
  int dof_qN;
  double rhoN;
  double T;
  double mo;  // R h / 6 of the edge (its end flux's lumped mass is R h / 2)

  __device__ __forceinline__ void setup(const PcArgs& pa, int c, bool active) {
    const int N = pa.N;
    const int l = threadIdx.x & (W - 1);
    const int e = active ? pa.chain_edge[c] : 0;
    const int flip = active ? pa.chain_flip[c] : 0;
    const int base = e * (2 * N + 1);
    const double* dqe = pa.dq + (int64_t)e * (N + 1);
    mo = active ? dqe[0] / pa.mo_div : 1.0;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      const int k = l * CPL + t;
      valid[t] = active && k < N;
      const int kp = flip ? N - 1 - k : k;
      const int qp = flip ? N - k : k;
      dof_c[t] = base + 2 * kp + 1;
      dof_q[t] = base + 2 * qp;
      rho[t] = valid[t] ? dqe[qp] : 0.0;
    }
    has_last = active && (l == (N - 1) / CPL);
    dof_qN = base + 2 * (flip ? 0 : N);
    rhoN = has_last ? dqe[flip ? 0 : N] : 0.0;
    finish();
  }

  // resistance distances and the chain total from rho / rhoN (k_dir_step sets those from
  // the masses it just assembled: the same bits as setup's loads of dq)
  __device__ __forceinline__ void finish() {
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      acc += rho[t];
      D[t] = acc;
    }
    const double excl = seg_incl_scan<W>(acc) - acc;
#pragma unroll
    for (int t = 0; t < CPL; ++t) D[t] += excl;
    T = seg_sum<W>(acc + rhoN);
  }
};

// Flux block of P^{-1} on the block's current chains: z_q = r_q / rho (lumped D) or, exact,
// z_q = M_e^{-1} r_q = T^{-1} r_q / mo by the Thomas algorithm run as two segment scans of
// affine maps (T = L U with pivots fixed by N: forward y_k = r_k - l_k y_{k-1}, backward
// x_k = (y_k - x_{k+1}) / u_k; pa.Tlu = [l_0..l_N | 1/u_0..1/u_N], l_0 = 0). T is
// persymmetric, so the chain direction (flip) does not matter. rq[t] is the lane's r at
// chain flux k = l CPL + t, rqN at q_N (the has_last lane, right after its last cell's
// flux). No LDS, no barriers; returns the lane's share of r . z.
// M_e^{-1} r on the lane's elements (its cells' fluxes, then q_N on the has_last lane) by
// the Thomas algorithm run as two segment scans of affine maps (T = L U with pivots fixed
// by N: forward y_k = r_k - l_k y_{k-1}, backward x_k = (y_k - x_{k+1}) / u_k; pa.Tlu =
// [l_0..l_N | 1/u_0..1/u_N], l_0 = 0); T is persymmetric, so the chain direction (flip)
// does not matter. out[t] = the solution at element t (0 where the lane has none).
template <int W, int CPL>
__device__ __forceinline__ void chain_mass_solve(const PcArgs& pa, const ChainLane<W, CPL>& ch,
                                                 const double* rq, double rqN,
                                                 double (&out)[CPL + 1]) {
  constexpr int NE = CPL + 1;
  const int N = pa.N;
  const int l = lane_of<W>();
  const double* __restrict__ lu = pa.Tlu;
  bool on[NE];
  double v[NE], lk[NE], iu[NE];
#pragma unroll
  for (int t = 0; t < NE; ++t) {
    on[t] = t < CPL ? ch.valid[t] : ch.has_last;
    const int k = t < CPL ? l * CPL + t : N;
    v[t] = t < CPL ? rq[t] : rqN;
    lk[t] = on[t] ? lu[k] : 0.0;
    iu[t] = on[t] ? lu[N + 1 + k] : 0.0;
  }
  // forward: y_k = -l_k y_{k-1} + r_k; the lane's composite map, then an inclusive scan
  double A = 1.0, B = 0.0;
#pragma unroll
  for (int t = 0; t < NE; ++t)
    if (on[t]) {
      B = -lk[t] * B + v[t];
      A = -lk[t] * A;
    }
#pragma unroll
  for (int o = 1; o < W; o <<= 1) {
    const double Ap = __shfl_up(A, o, W), Bp = __shfl_up(B, o, W);
    if (l >= o) {
      B = A * Bp + B;
      A = A * Ap;
    }
  }
  double y = __shfl_up(B, 1, W);  // y at the end of the previous lane (0 before q_0)
  if (l == 0) y = 0.0;
#pragma unroll
  for (int t = 0; t < NE; ++t)
    if (on[t]) {
      y = -lk[t] * y + v[t];
      v[t] = y;
    }
  // backward: x_k = (y_k - x_{k+1}) / u_k; composite over the lane (last element first),
  // then a suffix scan across lanes
  A = 1.0;
  B = 0.0;
#pragma unroll
  for (int t = NE - 1; t >= 0; --t)
    if (on[t]) {
      B = iu[t] * (v[t] - B);
      A = -iu[t] * A;
    }
#pragma unroll
  for (int o = 1; o < W; o <<= 1) {
    const double An = __shfl_down(A, o, W), Bn = __shfl_down(B, o, W);
    if (l + o < W) {
      B = A * Bn + B;
      A = A * An;
    }
  }
  double x = __shfl_down(B, 1, W);  // x at the start of the next lane (0 after q_N)
  if (l == W - 1) x = 0.0;
  const double imo = 1.0 / ch.mo;
#pragma unroll
  for (int t = NE - 1; t >= 0; --t) {
    out[t] = 0.0;
    if (on[t]) {
      x = iu[t] * (v[t] - x);
      out[t] = x * imo;
    }
  }
}

// Flux block of P^{-1} on the block's current chains: z_q = r_q / rho (lumped D) or, exact,
// z_q = M_e^{-1} r_q = T^{-1} r_q / mo (chain_mass_solve). rq[t] is the lane's r at chain
// flux k = l CPL + t, rqN at q_N (the has_last lane, right after its last cell's flux). No
// LDS, no barriers; returns the lane's share of r . z.
template <int W, int CPL>
__device__ __forceinline__ double pc_flux_block(const PcArgs& pa, const ChainLane<W, CPL>& ch,
                                                const double* rq, double rqN,
                                                double* __restrict__ z) {
  double part = 0.0;
  if (!pa.exact) {
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      if (!ch.valid[t]) continue;
      const double zq = rq[t] / ch.rho[t];
      z[ch.dof_q[t]] = zq;
      part += rq[t] * zq;
    }
    if (ch.has_last) {
      const double zq = rqN / ch.rhoN;
      z[ch.dof_qN] = zq;
      part += rqN * zq;
    }
    return part;
  }
  double zv[CPL + 1];
  chain_mass_solve<W, CPL>(pa, ch, rq, rqN, zv);
#pragma unroll
  for (int t = CPL; t >= 0; --t) {
    const bool on = t < CPL ? ch.valid[t] : ch.has_last;
    if (on) {
      z[t < CPL ? ch.dof_q[t] : ch.dof_qN] = zv[t];
      part += (t < CPL ? rq[t] : rqN) * zv[t];
    }
  }
  return part;
}

template <int BS>
__device__ __forceinline__ void pc_eliminate(const PcArgs& pa, const double* __restrict__ y,
                                             int j) {
  const int pcn = pa.slot_pchain[j];
  double D = pcn >= 0 ? 1.0 / pa.chain_T[pcn] : 0.0;
  double J = y[pa.slot_lam[j]] + (pcn >= 0 ? pa.chain_Ib[pcn] : 0.0);
  for (int i = pa.slot_dc_off[j]; i < pa.slot_dc_off[j + 1]; ++i) {
    const int c = pa.slot_dc[i];
    const double g = 1.0 / pa.chain_T[c];
    J += pa.chain_It[c];
    const int lo = pa.chain_lo[c];
    if (lo >= 0) {
      const double Dl = pa.slot_D[lo];
      D += g * (1.0 - g / Dl);
      J += g * pa.slot_J[lo] / Dl;
    } else {
      D += g;
    }
  }
  pa.slot_D[j] = D;
  pa.slot_J[j] = J;
}

__device__ __forceinline__ double pc_backsub(const PcArgs& pa, double* __restrict__ z, int j) {
  const int p = pa.slot_parent[j];
  double num = pa.slot_J[j];
  if (p >= 0) num += z[pa.slot_lam[p]] / pa.chain_T[pa.slot_pchain[j]];
  const double zj = num / pa.slot_D[j];
  z[pa.slot_lam[j]] = zj;
  return zj;
}

// mode 0: Lanczos step (r' = y - (alpha/beta) r2 in place of y, then condense r');
// mode 1: start (condense y = b as is).
template <bool MULTI, int W, int CPL>
__global__ __launch_bounds__(kBlock) void k_pc_up(PcArgs pa, double* __restrict__ y,
                                                  const double* __restrict__ r2,
                                                  MrState* __restrict__ st,
                                                  MrState* __restrict__ other,
                                                  const double* __restrict__ partA, int nA,
                                                  const double* __restrict__ red, int mode) {
  double c2 = 0.0;
  if (mode == 0) {
    if (st->done) {
      if (blockIdx.x == 0 && threadIdx.x == 0) *other = *st;  // see k_mr_b
      return;
    }
    const double alfa = MULTI ? red[0] : block_allsum(partA, nA);
    c2 = alfa / st->beta;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->alfa = alfa;
      st->nb += 1;
    }
  }
  const int job = blockIdx.x;
  const int c0 = pa.job_chain_off[job], c1 = pa.job_chain_off[job + 1];
  constexpr int G = kBlock / W;  // chains per pass
  const int seg = threadIdx.x / W, l = threadIdx.x & (W - 1);
  for (int cb = c0; cb < c1; cb += G) {
    const int c = cb + seg;
    const bool active = c < c1;
    ChainLane<W, CPL> ch;
    ch.setup(pa, c, active);
    double sr = 0.0, srd = 0.0;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      if (!ch.valid[t]) continue;
      double rc = y[ch.dof_c[t]];
      if (mode == 0) {
        rc -= c2 * r2[ch.dof_c[t]];
        y[ch.dof_c[t]] = rc;
        y[ch.dof_q[t]] -= c2 * r2[ch.dof_q[t]];
      }
      sr += rc;
      srd += rc * ch.D[t];
    }
    if (mode == 0 && ch.has_last) y[ch.dof_qN] -= c2 * r2[ch.dof_qN];
    sr = seg_sum<W>(sr);
    srd = seg_sum<W>(srd);
    if (active && l == 0) {
      const double ib = srd / ch.T;
      pa.chain_T[c] = ch.T;
      pa.chain_Ib[c] = ib;
      pa.chain_It[c] = sr - ib;
    }
  }
  // junction levels of this job, deepest first
  const int lv0 = pa.job_lvl_off[job], lv1 = pa.job_lvl_off[job + 1];
  if (lv1 > lv0) {
    if (mode == 0) {
      for (int j = pa.lvl_slot_off[lv0] + threadIdx.x; j < pa.lvl_slot_off[lv1]; j += kBlock) {
        const int lam = pa.slot_lam[j];
        y[lam] -= c2 * r2[lam];
      }
    }
    __syncthreads();
    for (int lv = lv1 - 1; lv >= lv0; --lv) {
      for (int j = pa.lvl_slot_off[lv] + threadIdx.x; j < pa.lvl_slot_off[lv + 1]; j += kBlock)
        pc_eliminate<kBlock>(pa, y, j);
      __syncthreads();
    }
  }
}

constexpr int kTopThreads = 1024;

template <bool MULTI>
__global__ __launch_bounds__(kTopThreads) void k_pc_top(PcArgs pa, double* __restrict__ y,
                                                        const double* __restrict__ r2,
                                                        double* __restrict__ z,
                                                        const MrState* __restrict__ st,
                                                        const double* __restrict__ partA, int nA,
                                                        const double* __restrict__ red,
                                                        double* __restrict__ partB, int mode) {
  double c2 = 0.0;
  if (mode == 0) {
    if (st->done) return;
    const double alfa = MULTI ? red[0] : block_allsum<kTopThreads>(partA, nA);
    c2 = alfa / st->beta;
  }
  const int nl = pa.n_top_lvl;
  const int s0 = pa.top_lvl_off[0], s1 = pa.top_lvl_off[nl];
  if (mode == 0) {
    for (int j = s0 + threadIdx.x; j < s1; j += kTopThreads) {
      const int lam = pa.slot_lam[j];
      y[lam] -= c2 * r2[lam];
    }
  }
  __syncthreads();
  for (int lv = nl - 1; lv >= 0; --lv) {
    for (int j = pa.top_lvl_off[lv] + threadIdx.x; j < pa.top_lvl_off[lv + 1]; j += kTopThreads)
      pc_eliminate<kTopThreads>(pa, y, j);
    __syncthreads();
  }
  if (MULTI && pa.n_coarse > 0) {  // back-substitution after the exchange (k_pc_coarse)
    pc_coarse_partials<kTopThreads>(pa, s0, s1 - s0, pa.slot_D + s0, pa.slot_J + s0);
    return;
  }
  double part = 0.0;
  for (int lv = 0; lv < nl; ++lv) {
    for (int j = pa.top_lvl_off[lv] + threadIdx.x; j < pa.top_lvl_off[lv + 1]; j += kTopThreads)
      part += y[pa.slot_lam[j]] * pc_backsub(pa, z, j);
    __syncthreads();
  }
  block_sum_store_n<kTopThreads>(part, partB + pa.n_jobs);
}

template <bool MULTI, int W, int CPL>
__global__ __launch_bounds__(kBlock) void k_pc_down(PcArgs pa, const double* __restrict__ y,
                                                    double* __restrict__ z,
                                                    const MrState* __restrict__ st,
                                                    double* __restrict__ partB, int mode) {
  if (mode == 0 && st->done) return;
  const int job = blockIdx.x;
  double part = 0.0;
  const int lv0 = pa.job_lvl_off[job], lv1 = pa.job_lvl_off[job + 1];
  for (int lv = lv0; lv < lv1; ++lv) {
    for (int j = pa.lvl_slot_off[lv] + threadIdx.x; j < pa.lvl_slot_off[lv + 1]; j += kBlock)
      part += y[pa.slot_lam[j]] * pc_backsub(pa, z, j);
    __syncthreads();
  }
  const int c0 = pa.job_chain_off[job], c1 = pa.job_chain_off[job + 1];
  constexpr int G = kBlock / W;
  const int seg = threadIdx.x / W;
  for (int cb = c0; cb < c1; cb += G) {
    const int c = cb + seg;
    const bool active = c < c1;
    ChainLane<W, CPL> ch;
    ch.setup(pa, c, active);
    const int up = active ? pa.chain_up[c] : -1, lo = active ? pa.chain_lo[c] : -1;
    const double zt = up >= 0 ? z[pa.slot_lam[up]] : 0.0;
    const double zb = lo >= 0 ? z[pa.slot_lam[lo]] : 0.0;
    const double T = ch.T, iT = 1.0 / T;
    double rc[CPL], a[CPL], b[CPL], rq[CPL];
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      rc[t] = ch.valid[t] ? y[ch.dof_c[t]] : 0.0;
      a[t] = (T - ch.D[t]) * rc[t];  // suffix sums over j >= k
      b[t] = ch.D[t] * rc[t];        // prefix sums over j < k
      sa += a[t];
      sb += b[t];
    }
    const double ia = seg_incl_scan<W>(sa), ib = seg_incl_scan<W>(sb);
    const double Atot = seg_sum<W>(sa);
    double pa_ = ia - sa, pb_ = ib - sb;  // exclusive lane carries
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      pa_ += a[t];  // inclusive prefix of a up to k
      const double suffix = Atot - pa_ + a[t];
      const double prefix = pb_;  // sum_{j<k} b_j
      pb_ += b[t];
      rq[t] = 0.0;
      if (!ch.valid[t]) continue;
      const double Dk = ch.D[t];
      double zk = zt * (T - Dk) * iT + zb * Dk * iT + Dk * iT * suffix + (T - Dk) * iT * prefix;
      if (pa.exact) zk -= ch.mo * rc[t];
      z[ch.dof_c[t]] = zk;
      part += rc[t] * zk;
      rq[t] = y[ch.dof_q[t]];
    }
    const double rqN = ch.has_last ? y[ch.dof_qN] : 0.0;
    part += pc_flux_block<W, CPL>(pa, ch, rq, rqN, z);
  }
  block_sum_store(part, partB + blockIdx.x);
}

// ---- LDS variants: one 1024-thread workgroup per job, the junction levels run in LDS.
// Phase A gathers, in one parallel pass, every static index and every chain result a
// junction needs (own parent chain, chains hanging below, children as local LDS indices);
// phase B sweeps the levels touching LDS only. The host picks these kernels when every
// job fits the caps below (always for the binary / arterial trees), else the global ones.
constexpr int kPcThreads = 1024;
constexpr int kCapC = 512;    // chains per job
constexpr int kCapS = 256;    // junction slots per job
constexpr int kCapDC = 768;   // down-chain entries per job
constexpr int kCapT = 1152;   // top junction slots (host caps the top part at 1024)
constexpr int kCapTDC = 2304; // top down-chain entries
constexpr int kMaxTopLvl = 255;
constexpr int kMaxNeed = 128;  // dense top: top values one job reads (precond.K_MAX_NEED)

__device__ void pc_cpart_last(const PcArgs& pa, double* sA);

// Direct solve (nx_set_solver; mode kModeDirect of the LDS sweeps, one rank): the sweeps
// apply S^{-1} to w = K^T M^{-1} b_q - b_s and finish x_q = M^{-1} (b_q - K x_s) themselves.
constexpr int kModeDirect = 3;

// Cell inputs of one chain for the direct solve: y = M^{-1} b_q (Thomas scans), then
// w_c = (K^T y)_c - b_c in place of vc (row p_g of the layout: +q_g - q_{g+1}; cell k of the
// chain lies between chain fluxes k and k + 1, whose orientation flips the sign). ytop / ybot
// (valid in every lane): the multiplier rows' K^T y at the chain's top / bottom end -- the
// layout puts -1 at q_0 (source multiplier) and +1 at q_N (target multiplier).
template <int W, int CPL>
__device__ __forceinline__ void direct_cell_inputs(const PcArgs& pa, const ChainLane<W, CPL>& ch,
                                                   int flip, const double* bq, double bqN,
                                                   double* vc, double& ytop, double& ybot) {
#pragma clang fp contract(off)
  double yv[CPL + 1];
  chain_mass_solve<W, CPL>(pa, ch, bq, bqN, yv);
  const int N = pa.N;
  const int l = lane_of<W>();
  const double nxt0 = __shfl_down(yv[0], 1, W);
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    const int k = l * CPL + t;
    const double ynext = (k + 1 == N) ? yv[CPL] : (t + 1 < CPL ? yv[t + 1] : nxt0);
    const double d = yv[t] - ynext;
    vc[t] = ch.valid[t] ? (flip ? -d : d) - vc[t] : 0.0;
  }
  const double y0 = __shfl(yv[0], 0, W), yN = __shfl(yv[CPL], (N - 1) / CPL, W);
  ytop = flip ? y0 : -y0;  // top = chain position 0 = the edge's source unless flipped
  ybot = flip ? -yN : yN;
}

// Fluxes of one chain from its end and cell values, conservatively: x_q = M^{-1}(b_q - K x_s)
// computed flux by flux takes differences of neighbouring pressures, whose rounding
// (eps |p|) divided by the cell mass R h leaves the divergence rows a residual of
// eps |p| / (R h) -- 1e-11 relative on the depth-17 tree. The exact solution satisfies the N
// divergence rows exactly, so they fix every flux from the first one,
//   x_q[k] = q_0 - s P_k,   P_k = sum_{j<k} b_c[j]   (s = -1 on a flipped chain),
// and the d-weighted sum of the N + 1 flux rows (1^T M = d^T, d = lumped mass; 1^T K x_s
// telescopes to s (z_bot - z_top)) fixes q_0:
//   T q_0 = sum_k b_q[k] - s (z_bot - z_top) + s sum_k d_k P_k,   T = sum_k d_k.
// Same solution in exact arithmetic; the divergence rows' residual is then exactly zero and
// the flux / multiplier rows' stays at eps |p| (one pass: 2.9e-13 -> 3e-14 at C3).
// bc / bq: the lane's b at its cells / fluxes (chain order), bqN at q_N (has_last lane).
template <int W, int CPL>
__device__ __forceinline__ void direct_flux_cons(const ChainLane<W, CPL>& ch, int flip,
                                                 const double* bc, const double* bq, double bqN,
                                                 double zt, double zb, double (&out)[CPL + 1]) {
#pragma clang fp contract(off)
  const int l = lane_of<W>();
  double loc = 0.0;
#pragma unroll
  for (int t = 0; t < CPL; ++t)
    if (ch.valid[t]) loc += bc[t];
  const double incl = seg_incl_scan<W>(loc);
  double run = __shfl_up(incl, 1, W);  // cells before this lane's first
  if (l == 0) run = 0.0;
  double P[CPL + 1];
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    P[t] = run;
    if (ch.valid[t]) {
      s1 += bq[t];
      s2 += ch.rho[t] * run;
      run += bc[t];
    }
  }
  P[CPL] = run;  // q_N (the has_last lane holds cell N - 1): every cell
  if (ch.has_last) {
    s1 += bqN;
    s2 += ch.rhoN * run;
  }
  s1 = seg_sum<W>(s1);
  s2 = seg_sum<W>(s2);
  const double sg = flip ? -1.0 : 1.0;
  const double q0 = (s1 - sg * (zb - zt) + sg * s2) / ch.T;
#pragma unroll
  for (int t = 0; t < CPL; ++t) out[t] = ch.valid[t] ? q0 - sg * P[t] : 0.0;
  out[CPL] = ch.has_last ? q0 - sg * P[CPL] : 0.0;
}

// mo = R h / 6 of the lane's cells (chain order), with k_assemble's arithmetic: the CSR
// values are R h / 3 and R h / 6 of the same h, bit for bit (direct_residual).
template <int W, int CPL>
__device__ __forceinline__ void chain_cell_mo(const PcArgs& pa, const ChainLane<W, CPL>& ch, int c,
                                              bool active, int flip, double* mo) {
#pragma clang fp contract(off)
  const int N = pa.N;
  const int l = threadIdx.x & (W - 1);
  const int e = active ? pa.chain_edge[c] : 0;
  double x0[3], x1[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    x0[i] = pa.edge_x[6 * (int64_t)e + i];
    x1[i] = pa.edge_x[6 * (int64_t)e + 3 + i];
  }
  const double R = pa.edge_R[e];
  const double invN = pa.invN;
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    mo[t] = 0.0;
    if (!ch.valid[t]) continue;
    const int k = l * CPL + t;
    const int kp = flip ? N - 1 - k : k;  // the edge's cell
    double va[3], vb[3];
    vertex(x0, x1, kp, N, invN, va);
    vertex(x0, x1, kp + 1, N, invN, vb);
    const double d0 = vb[0] - va[0], d1 = vb[1] - va[1], d2 = vb[2] - va[2];
    const double h = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
    mo[t] = R * h / 6.0;
  }
}

// The direct solve's true residual on one chain's rows, r = vin - A out (pa.fres): vin = the
// sweeps' input (b; the previous residual in a refinement pass, r' = r - A d), out = their
// output (x; the correction d) -- cells xc, fluxes xq (q_N in xq[CPL] of the has_last lane),
// end junctions zt / zb. The operator is the assembled one: the cell masses R h / 3, R h / 6
// are regenerated with k_assemble's arithmetic (bit-identical CSR values), the pressure and
// multiplier couplings are +-1 (k_pattern's rows, chain order: s = -1 on a flipped chain).
// Stores r, adds r^2 and vin^2 to rr / bb, and posts the chain's shares of its end junctions'
// multiplier rows (A[lam_top, q_0] = -s, A[lam_bot, q_N] = +s) to sQt / sQb[lc].
template <int W, int CPL, bool STORE = true>
__device__ __forceinline__ void direct_residual(const PcArgs& pa, const ChainLane<W, CPL>& ch,
                                                bool active, int flip, const double* vc,
                                                const double* vq, double vqN, const double* xc,
                                                const double (&xq)[CPL + 1], double zt, double zb,
                                                const double* mo, double& rr, double& bb,
                                                double* sQt, double* sQb, int lc) {
#pragma clang fp contract(off)
  const int N = pa.N;
  const int l = lane_of<W>();
  const double sg = flip ? -1.0 : 1.0;
  // md = R h / 3 = 2 mo exactly (mo = R h / 6: halving is exact in binary)
  double md[CPL];
#pragma unroll
  for (int t = 0; t < CPL; ++t) md[t] = 2.0 * mo[t];
  // cell k - 1 of element 0 and flux k + 1 of the last element live in the neighbour lanes
  const double mdP = __shfl_up(md[CPL - 1], 1, W), moP = __shfl_up(mo[CPL - 1], 1, W);
  const double xcP = __shfl_up(xc[CPL - 1], 1, W), xqP = __shfl_up(xq[CPL - 1], 1, W);
  const double xqX = __shfl_down(xq[0], 1, W);
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    if (!ch.valid[t]) continue;
    const int k = l * CPL + t;
    const double qn = (k + 1 == N) ? xq[CPL] : (t + 1 < CPL ? xq[t + 1] : xqX);
    const double rc = vc[t] - sg * (xq[t] - qn);  // cell row: s (q_k - q_{k+1})
    double acc, xcl;
    if (k == 0) {
      acc = md[t] * xq[t] + mo[t] * qn;
      xcl = zt;
    } else {
      const double mdl = t > 0 ? md[t - 1] : mdP, mol = t > 0 ? mo[t - 1] : moP;
      const double xql = t > 0 ? xq[t - 1] : xqP;
      xcl = t > 0 ? xc[t - 1] : xcP;
      acc = mol * xql + (mdl + md[t]) * xq[t] + mo[t] * qn;
    }
    const double rq = vq[t] - (acc + sg * (xc[t] - xcl));  // flux row: mass + s (p_k - p_{k-1})
    if (STORE) {  // (a refinement step starts from r; k_dir_step does not keep it)
      pa.rres[ch.dof_c[t]] = rc;
      pa.rres[ch.dof_q[t]] = rq;
    }
    rr += rc * rc + rq * rq;
    bb += vc[t] * vc[t] + vq[t] * vq[t];
  }
  if (ch.has_last) {  // q_N: cell N - 1 and the bottom junction
    const int tl = (N - 1) - l * CPL;
    double mdl = 0.0, mol = 0.0, xql = 0.0, xcl = 0.0;
#pragma unroll
    for (int t = 0; t < CPL; ++t)
      if (t == tl) {
        mdl = md[t];
        mol = mo[t];
        xql = xq[t];
        xcl = xc[t];
      }
    const double rq = vqN - ((mol * xql + mdl * xq[CPL]) + sg * (zb - xcl));
    if (STORE) pa.rres[ch.dof_qN] = rq;
    rr += rq * rq;
    bb += vqN * vqN;
    sQb[lc] = sg * xq[CPL];
  }
  if (l == 0 && active) sQt[lc] = -sg * xq[0];
}

constexpr int kCapLvl = 64;  // job levels whose slot offsets are staged in LDS
constexpr int kWaveKids = 4;  // junction children per slot of the one-wave level sweeps

template <bool MULTI, int W, int CPL>
__global__ __launch_bounds__(kPcThreads) void k_pc_up_lds(PcArgs pa, double* __restrict__ y,
                                                          const double* __restrict__ r2,
                                                          MrState* __restrict__ st,
                                                          MrState* __restrict__ other,
                                                          const double* __restrict__ partA,
                                                          int nA, const double* __restrict__ red,
                                                          int mode) {
  __shared__ double sT[kCapC], sIt[kCapC], sIb[kCapC];
  __shared__ double sD0[kCapS], sJ0[kCapS], sD[kCapS], sJ[kCapS];
  __shared__ double sIv[kCapS];  // direct mode: 1 / D of every slot (one division per slot)
  __shared__ int sChild[kCapDC];
  __shared__ double sG[kCapDC];
  __shared__ int sOff[kCapS + 1];
  __shared__ int sLvl[kCapLvl + 1];
  __shared__ double sAtop[MULTI ? kCapT : 1];  // fused k_pc_cpart (last workgroup)
  double c2 = 0.0;
  // alpha's partials first: their loads overlap the state read and the prefetch below
  const double pA = mode == 0 && !MULTI ? block_partial<kPcThreads>(partA, nA) : 0.0;
  const bool upd = mode == 0 && !(MULTI && pa.lin);
  // direct solve (mode 3): y holds b; the chains condense w = K^T M^{-1} b_q - b
  // (formed here from b) and their It / Ib carry the multiplier rows' share of K^T M^{-1} b_q
  const bool dir = mode == kModeDirect;
  const int job = blockIdx.x;
  const int c0 = pa.job_chain_off[job], c1 = pa.job_chain_off[job + 1];
  constexpr int G = kPcThreads / W;
  const int seg = threadIdx.x / W, l = threadIdx.x & (W - 1);
  // prefetch, independent of alpha (its re-reduction below hides the latency): the first
  // chain pass's lane setup and values, and this thread's junction slot of phase A
  ChainLane<W, CPL> ch;
  ch.setup(pa, c0 + seg, c0 + seg < c1);
  double vc[CPL], wc[CPL], vq[CPL], wq[CPL], vN = 0.0, wN = 0.0;
  int flip = 0;
  auto load_lane = [&](int c, bool active) {
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      vc[t] = ch.valid[t] ? y[ch.dof_c[t]] : 0.0;
      wc[t] = upd && ch.valid[t] ? r2[ch.dof_c[t]] : 0.0;
      vq[t] = (upd || dir) && ch.valid[t] ? y[ch.dof_q[t]] : 0.0;
      wq[t] = upd && ch.valid[t] ? r2[ch.dof_q[t]] : 0.0;
    }
    vN = (upd || dir) && ch.has_last ? y[ch.dof_qN] : 0.0;
    wN = upd && ch.has_last ? r2[ch.dof_qN] : 0.0;
    flip = dir && active ? pa.chain_flip[c] : 0;
  };
  load_lane(c0 + seg, c0 + seg < c1);
  const int lv0 = pa.job_lvl_off[job], lv1 = pa.job_lvl_off[job + 1];
  const int js0 = lv1 > lv0 ? pa.lvl_slot_off[lv0] : 0;
  const int js1 = lv1 > lv0 ? pa.lvl_slot_off[lv1] : 0;
  const bool fac = pa.factored && mode == 0;
  constexpr int kPre = 4;  // down-chain entries of the slot prefetched
  int p_lam = 0, p_pcn = -1, p_o0 = 0, p_o1 = 0, p_dc[kPre], p_lo[kPre];
  double p_y = 0.0, p_r = 0.0, p_kap[kPre];
  if ((int)threadIdx.x < js1 - js0) {
    const int j = js0 + threadIdx.x;
    p_lam = pa.slot_lam[j];
    p_pcn = pa.slot_pchain[j];
    p_o0 = pa.slot_dc_off[j];
    p_o1 = pa.slot_dc_off[j + 1];
    p_y = y[p_lam];
    p_r = upd ? r2[p_lam] : 0.0;
#pragma unroll
    for (int q = 0; q < kPre; ++q) {
      const bool in = p_o0 + q < p_o1;
      p_dc[q] = in ? pa.slot_dc[p_o0 + q] : 0;
      p_lo[q] = in ? pa.dc_lo[p_o0 + q] : -1;
      p_kap[q] = in && fac ? pa.dc_kappa[p_o0 + q] : 0.0;
    }
  }
  // the stop test after the prefetch: its load no longer delays the loads above (they are
  // harmless when the solve has stopped; nothing is written before this point)
  if (mode == 0 && st->done) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *other = *st;  // see k_mr_b
    return;
  }
  if (mode == 0 && !(MULTI && pa.lin)) {  // linear form: alpha is not known yet (k_pc_coarse)
    const double alfa = MULTI ? red[0] : block_allsum_v<kPcThreads>(pA);
    c2 = alfa / st->beta;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->alfa = alfa;
      st->nb += 1;
    }
  }
  if (MULTI && pa.lin && mode == 0 && blockIdx.x == 0) {  // this rank's alpha partial sum
    const double a = block_allsum<kPcThreads>(partA, nA);
    if (threadIdx.x == 0) const_cast<double*>(pa.xalpha)[0] = a;
  }
  const bool dense = (MULTI ? pa.mdense : pa.dense) && mode == 0;  // write the top inputs u
  NX_PHASE_START(16);
  for (int cb = c0; cb < c1; cb += G) {
    const int c = cb + seg;
    const bool active = c < c1;
    if (cb != c0) {  // more chains than one pass: set up and load here
      ch.setup(pa, c, active);
      load_lane(c, active);
    }
    double ytop = 0.0, ybot = 0.0;
    if (dir) direct_cell_inputs<W, CPL>(pa, ch, flip, vq, vN, vc, ytop, ybot);
    double sr = 0.0, srd = 0.0;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      if (!ch.valid[t]) continue;
      double rc = vc[t];
      if (upd) {
        rc -= c2 * wc[t];
        y[ch.dof_c[t]] = rc;
        y[ch.dof_q[t]] = vq[t] - c2 * wq[t];
      }
      sr += rc;
      srd += rc * ch.D[t];
    }
    if (upd && ch.has_last) y[ch.dof_qN] = vN - c2 * wN;
    sr = seg_sum<W>(sr);
    srd = seg_sum<W>(srd);
    if (active && l == 0) {
      const double ib = srd / ch.T;
      const double it = (sr - ib) + ytop, ibe = ib + ybot;  // dir: + the multiplier rows' share
      sT[c - c0] = ch.T;
      sIb[c - c0] = dir ? ibe : ib;
      sIt[c - c0] = dir ? it : sr - ib;
      pa.chain_T[c] = ch.T;
      pa.chain_Ib[c] = dir ? ibe : ib;
      pa.chain_It[c] = dir ? it : sr - ib;
      if (dense) {
        const int ui = pa.chain_uit[c], ub = pa.chain_uib[c];
        if (ui >= 0) pa.u[ui] = sr - ib;
        if (ub >= 0) pa.u[ub] = ib;
      }
    }
  }
  NX_PHASE(17);
  if (dense) {  // the top kernel does not run: update the job's top rows, post their y'
    const int ts0 = pa.top_lvl_off[0];
    for (int i = pa.job_tslot_off[job] + threadIdx.x; i < pa.job_tslot_off[job + 1]; i += kPcThreads) {
      const int t = pa.job_tslot[i];
      const int lam = pa.slot_lam[t];
      const double yl = y[lam] - c2 * r2[lam];
      y[lam] = yl;
      pa.u[pa.slot_uy[t - ts0]] = yl;
    }
  }
  // the host-built one-wave set-up of this job's levels (loaded here, used after phase A)
  const int jwave = (lv1 > lv0 && pa.job_wave) ? pa.job_wave[job] : 0;
  int wv0 = 0, wv1 = 0, wv2 = 0;
  if (jwave > 0 && (int)threadIdx.x < js1 - js0) {
    const int* w = pa.slot_wave + 3 * (int64_t)(js0 + threadIdx.x);
    wv0 = w[0];
    wv1 = w[1];
    wv2 = w[2];
  }
  if (lv1 > lv0) {  // the job's junction levels (block-uniform)
  const int ns = js1 - js0;
  const int dc0 = pa.slot_dc_off[js0];
  // factored: D is fixed by the assembly -> J += kappa J_child, no divisions, no D stores
  __syncthreads();
  for (int sl = threadIdx.x; sl < ns; sl += kPcThreads) {  // phase A
    const int j = js0 + sl;
    const bool pre = sl == (int)threadIdx.x;  // the prefetched slot
    const int lam = pre ? p_lam : pa.slot_lam[j];
    double yl = pre ? p_y : y[lam];
    if (upd) {
      yl -= c2 * (pre ? p_r : r2[lam]);
      y[lam] = yl;
    }
    if (dir) yl = -yl;  // w_lambda = (K^T M^{-1} b_q)_lambda - b_lambda; the first part is in It / Ib
    const int pcn = pre ? p_pcn : pa.slot_pchain[j];
    double D0 = pcn >= 0 ? 1.0 / sT[pcn - c0] : 0.0;
    double J0 = yl + (pcn >= 0 ? sIb[pcn - c0] : 0.0);
    const int o0 = pre ? p_o0 : pa.slot_dc_off[j], o1 = pre ? p_o1 : pa.slot_dc_off[j + 1];
    sOff[sl] = o0 - dc0;
    for (int i = o0; i < o1; ++i) {
      const int q = i - o0;
      const bool pq = pre && q < kPre;
      int dcq = 0, loq = -1;
      double kq = 0.0;
#pragma unroll
      for (int r = 0; r < kPre; ++r)
        if (r == q) {
          dcq = p_dc[r];
          loq = p_lo[r];
          kq = p_kap[r];
        }
      const int cl = (pq ? dcq : pa.slot_dc[i]) - c0;
      const int lo = pq ? loq : pa.dc_lo[i];
      const double g = 1.0 / sT[cl];
      J0 += sIt[cl];
      if (lo >= 0) {
        sChild[i - dc0] = lo - js0;
        sG[i - dc0] = fac ? (pq ? kq : pa.dc_kappa[i]) : g;
      } else {
        sChild[i - dc0] = -1;
        D0 += g;
      }
    }
    sD0[sl] = D0;
    sJ0[sl] = J0;
  }
  if (threadIdx.x == 0) sOff[ns] = pa.slot_dc_off[js1] - dc0;
  if ((int)threadIdx.x <= min(lv1 - lv0, kCapLvl)) sLvl[threadIdx.x] = pa.lvl_slot_off[lv0 + threadIdx.x];
  __syncthreads();
  NX_PHASE(18);
  // phase B by one wave when the job has <= 64 slots with <= kWaveKids junction children
  // each (every job of the binary trees): lane = slot, the children's values by shuffles,
  // no workgroup barrier per level (~0.5 us each). Same arithmetic in the same order.
  bool wave_lv = jwave > 0;  // host-built set-up (pa.slot_wave)
  if (!wave_lv) {
    int nkids = 0;
    if ((int)threadIdx.x < ns)
      for (int i = sOff[threadIdx.x]; i < sOff[threadIdx.x + 1]; ++i) nkids += sChild[i] >= 0;
    wave_lv = __syncthreads_or(nkids > kWaveKids) == 0 && ns <= 64 && lv1 - lv0 <= kCapLvl;
  }
  if (wave_lv) {
    if (threadIdx.x < 64) {
      const int sl = threadIdx.x;
      const bool mine = sl < ns;
      int mylv = -1;
      int cl[kWaveKids];
      double cg[kWaveKids];
#pragma unroll
      for (int k = 0; k < kWaveKids; ++k) {
        cl[k] = sl;
        cg[k] = 0.0;
      }
      int nk = 0, kmax;
      if (jwave > 0) {  // level, children and their dc entries from the host
        kmax = jwave - 1;
        if (mine) {
          mylv = wv0 & 0xff;
          nk = (wv0 >> 8) & 0xff;
          const int cw[kWaveKids] = {wv1 & 0xffff, wv1 >> 16, wv2 & 0xffff, wv2 >> 16};
#pragma unroll
          for (int k = 0; k < kWaveKids; ++k)
            if (k < nk) {
              cl[k] = cw[k] & 63;
              cg[k] = sG[cw[k] >> 6];
            }
        }
      } else {
        for (int q = 0; q < lv1 - lv0; ++q)
          if (mine && js0 + sl >= sLvl[q] && js0 + sl < sLvl[q + 1]) mylv = q;
        if (mine)
          for (int i = sOff[sl]; i < sOff[sl + 1]; ++i) {
            const int chd = sChild[i];
            if (chd < 0) continue;
#pragma unroll
            for (int k = 0; k < kWaveKids; ++k)
              if (k == nk) {
                cl[k] = chd;
                cg[k] = sG[i];
              }
            ++nk;
          }
        kmax = nk;
        for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o));
      }
      double D = mine ? sD0[sl] : 1.0, J = mine ? sJ0[sl] : 0.0, iv = 1.0;
#ifdef NX_PHASE_TIMING
      if (blockIdx.x == 0 && threadIdx.x == 0) g_phase[21] = wall_clock64();  // setup done
#endif
      for (int q = lv1 - lv0 - 1; q >= 0; --q) {
#pragma unroll
        for (int k = 0; k < kWaveKids; ++k) {
          if (k >= kmax) break;
          const double Jc = __shfl(J, cl[k]);
          const double Dc = __shfl(dir ? iv : D, cl[k]);
          if (mylv == q && k < nk) {
            const double g = cg[k];
            if (fac) {
              J += g * Jc;
            } else if (dir) {
              D += g * (1.0 - g * Dc);
              J += g * Jc * Dc;
            } else {
              D += g * (1.0 - g / Dc);
              J += g * Jc / Dc;
            }
          }
        }
        if (dir && mylv == q) iv = 1.0 / D;
      }
      if (mine) {
        sD[sl] = D;
        sJ[sl] = J;
        if (dir) sIv[sl] = iv;
      }
    }
    __syncthreads();
  } else
  for (int lv = lv1 - 1; lv >= lv0; --lv) {  // phase B, deepest level first
    // level offsets staged in LDS with phase A (a global load per level costs a round trip)
    const int la = lv - lv0 <= kCapLvl ? sLvl[lv - lv0] : pa.lvl_slot_off[lv];
    const int lb = lv - lv0 < kCapLvl ? sLvl[lv - lv0 + 1] : pa.lvl_slot_off[lv + 1];
    for (int j = la + threadIdx.x; j < lb; j += kPcThreads) {
      const int sl = j - js0;
      double D = sD0[sl], J = sJ0[sl];
      if (fac) {
        for (int i = sOff[sl]; i < sOff[sl + 1]; ++i) {
          const int ch = sChild[i];
          if (ch >= 0) J += sG[i] * sJ[ch];
        }
      } else if (dir) {  // the children's 1 / D: no division on the level's critical path
        for (int i = sOff[sl]; i < sOff[sl + 1]; ++i) {
          const int ch = sChild[i];
          if (ch < 0) continue;
          const double g = sG[i], iv = sIv[ch];
          D += g * (1.0 - g * iv);
          J += g * sJ[ch] * iv;
        }
        sIv[sl] = 1.0 / D;
      } else {
        for (int i = sOff[sl]; i < sOff[sl + 1]; ++i) {
          const int ch = sChild[i];
          if (ch < 0) continue;
          const double g = sG[i], Dc = sD[ch];
          D += g * (1.0 - g / Dc);
          J += g * sJ[ch] / Dc;
        }
      }
      sD[sl] = D;
      sJ[sl] = J;
    }
    __syncthreads();
  }
  NX_PHASE(20);
  for (int sl = threadIdx.x; sl < ns; sl += kPcThreads) {
    const int j = js0 + sl;
    const double J = sJ[sl];
    pa.slot_J[j] = J;
    if (fac) {
      pa.slot_A[j] = J * pa.slot_invD[j];
    } else if (dir) {
      const int pcn = pa.slot_pchain[j];
      const double iv = sIv[sl];
      pa.slot_D[j] = sD[sl];
      pa.slot_A[j] = J * iv;
      pa.slot_B[j] = pcn >= 0 ? iv / sT[pcn - c0] : 0.0;
    } else {
      const int pcn = pa.slot_pchain[j];
      const double D = sD[sl];
      pa.slot_D[j] = D;
      pa.slot_A[j] = J / D;
      pa.slot_B[j] = pcn >= 0 ? 1.0 / (sT[pcn - c0] * D) : 0.0;
    }
  }
  if (dense && threadIdx.x == 0 && pa.job_root_u[job] >= 0) {  // root -> its top parent
    const int k = pa.job_root_dc[job];
    const int pcn = pa.slot_pchain[js0];
    const double kap = fac ? pa.dc_kappa[k] : 1.0 / sT[pcn - c0] / sD[0];
    pa.u[pa.job_root_u[job]] = sIt[pcn - c0] + kap * sJ[0];
  }
  }  // junction levels
  NX_PHASE(19);
  NX_PHASE_END(16);
  if (MULTI && dense && pa.fused) pc_cpart_last(pa, sAtop);
}

// LDS of the top part's solve (k_pc_top_lds; with pa.topdown also every direct down sweep)
struct TopLds {
  double *sD0, *sJ0, *sD, *sJ, *sGp, *sY;
  int *sPar, *sLam, *sOff, *sChild;
  double *sG, *sDD, *sDJ;
  int* sLv;
};

// This thread's first entries of the top part's phases A1 (hanging chain tid) and A2 (slot
// tid): indices (top_pre_idx, one round trip: the top part's extent is host-known, PcArgs
// top_*) and the values they point at (top_pre_val, one more), so a caller can issue both
// among its own loads (the direct down sweep: beside its chain prefetch).
struct TopPre {
  int c, lo, lam, pcn, par, off;
  double T, It, Dl, Jl, y, Tp, Ib;
  int w[1 + kWaveKids];  // pa.top_wave (or top_sub) of slot tid (loaded with the indices)
  int ls, lw[1 + kWaveKids], ldep;  // pa.top_lane of thread tid, its wave's subtree depth
};

__device__ __forceinline__ void top_pre_idx(const PcArgs& pa, TopPre& p) {
  const int tid = threadIdx.x;
  const int ts0 = pa.top_ts0, nt = pa.top_nt, dc0 = pa.top_dc0, ndc = pa.top_ndc;
  p.c = tid < ndc ? pa.slot_dc[dc0 + tid] : 0;
  p.lo = tid < ndc ? pa.dc_lo[dc0 + tid] : -1;
  p.lam = tid < nt ? pa.slot_lam[ts0 + tid] : 0;
  p.pcn = tid < nt ? pa.slot_pchain[ts0 + tid] : -1;
  p.par = tid < nt ? pa.slot_parent[ts0 + tid] : -1;
  p.off = tid < nt ? pa.slot_dc_off[ts0 + tid] : 0;
  const int* tw = pa.top_sub ? pa.top_sub : pa.top_wave;
#pragma unroll
  for (int k = 0; k <= kWaveKids; ++k)
    p.w[k] = (tw && tid < nt) ? tw[(1 + kWaveKids) * (int64_t)tid + k] : 0;
  p.ls = -1;
  p.ldep = 0;
#pragma unroll
  for (int k = 0; k <= kWaveKids; ++k) p.lw[k] = 0;
  if (pa.top_sub) {
    const int* lt = pa.top_lane + (2 + kWaveKids) * (int64_t)tid;
    p.ls = lt[0];
#pragma unroll
    for (int k = 0; k <= kWaveKids; ++k) p.lw[k] = lt[1 + k];
    p.ldep = pa.top_sub_dep[tid >> 6];
  }
}

// WT: the inputs were handed over inside the launch (k_dir_step): write-through loads; y
// null: the multiplier rows' rhs is zero (the assembled b, first pass)
template <bool WT = false>
__device__ __forceinline__ void top_pre_val(const PcArgs& pa, const double* __restrict__ y,
                                            TopPre& p) {
  const int tid = threadIdx.x;
  const int ts0 = pa.top_ts0, ts1 = pa.top_ts0 + pa.top_nt;
  const bool dc = tid < pa.top_ndc, sl = tid < pa.top_nt;
  const bool low = dc && p.lo >= 0 && !(p.lo >= ts0 && p.lo < ts1);  // a lower job's root
  p.T = dc ? ldv<WT>(pa.chain_T + p.c) : 1.0;
  p.It = dc ? ldv<WT>(pa.chain_It + p.c) : 0.0;
  p.Dl = low ? ldv<WT>(pa.slot_D + p.lo) : 1.0;
  p.Jl = low ? ldv<WT>(pa.slot_J + p.lo) : 0.0;
  p.y = sl && y ? y[p.lam] : 0.0;
  p.Tp = sl && p.pcn >= 0 ? ldv<WT>(pa.chain_T + p.pcn) : 1.0;
  p.Ib = sl && p.pcn >= 0 ? ldv<WT>(pa.chain_Ib + p.pcn) : 0.0;
}

// The top part's elimination and back-substitution (one workgroup of kTopThreads). down = 1:
// run inside a direct down sweep (pa.topdown, one rank): the top values stay in LDS (sJ0)
// for the workgroup's own chains, workgroup 0 stores them in slot_z (k_dir_publish_fr moves
// them into x after the sweep), nothing else is written.
// WT (k_dir_step's last workgroup): the inputs come write-through (top_pre_val) and the
// values go out write-through (slot_z) to the other workgroups of the launch.
template <bool MULTI, bool WT = false>
__device__ __forceinline__ void top_body(const PcArgs& pa, double* __restrict__ y,
                                         const double* __restrict__ r2, double* __restrict__ z,
                                         const MrState* __restrict__ st,
                                         const double* __restrict__ partA, int nA,
                                         const double* __restrict__ red,
                                         double* __restrict__ partB, int mode, const TopLds& L,
                                         bool down, const TopPre& pre_in) {
  // no contraction: the kernel and every down workgroup (topdown) must agree bit for bit
#pragma clang fp contract(off)
  double *sD0 = L.sD0, *sJ0 = L.sJ0, *sD = L.sD, *sJ = L.sJ, *sGp = L.sGp, *sY = L.sY;
  int *sPar = L.sPar, *sLam = L.sLam, *sOff = L.sOff, *sChild = L.sChild;
  double *sG = L.sG, *sDD = L.sDD, *sDJ = L.sDJ;
  int* sLv = L.sLv;
  double c2 = 0.0;
  const bool upd = mode == 0 && !(MULTI && pa.lin);
  // the first pass of phases A1 / A2 comes prefetched (top_pre_idx / top_pre_val, issued
  // by the caller before the stop test and alpha's re-reduction)
  const int nl = pa.n_top_lvl;
  const int ts0 = pa.top_ts0, nt = pa.top_nt, ts1 = ts0 + nt;
  const int dc0 = pa.top_dc0, ndc = pa.top_ndc;
  const int tid = threadIdx.x;
  const TopPre& pre_ = pre_in;
  const int p_c = pre_.c, p_lo = pre_.lo, p_lam = pre_.lam, p_pcn = pre_.pcn, p_par = pre_.par,
            p_off = pre_.off;
  if (mode == 0) {
    if (st->done) return;
    if (upd) {
      const double alfa = MULTI ? red[0] : block_allsum<kTopThreads>(partA, nA);
      c2 = alfa / st->beta;
    }
  }
  NX_PHASE_START(32);
  for (int i = threadIdx.x; i <= nl; i += kTopThreads) sLv[i] = pa.top_lvl_off[i];
  // phase A1, one thread per hanging chain: its conductance, its top current and, for a
  // lower-job root below it (final Norton pair) or ground, its whole contribution
  for (int i = threadIdx.x; i < ndc; i += kTopThreads) {
    const bool pre = i == tid;
    const int c = pre ? p_c : pa.slot_dc[dc0 + i];
    const int lo = pre ? p_lo : pa.dc_lo[dc0 + i];
    const double g = 1.0 / (pre ? pre_.T : ldv<WT>(pa.chain_T + c));
    const double it = pre ? pre_.It : ldv<WT>(pa.chain_It + c);
    int child = -1;
    double dD = 0.0, dJ = it;
    if (lo >= ts0 && lo < ts1) {  // child above the cut: solved in the level sweep
      child = lo - ts0;
    } else if (lo >= 0) {
      const double Dl = pre ? pre_.Dl : ldv<WT>(pa.slot_D + lo);
      dD = g * (1.0 - g / Dl);
      dJ += g * (pre ? pre_.Jl : ldv<WT>(pa.slot_J + lo)) / Dl;
    } else {
      dD = g;
    }
    sChild[i] = child;
    sG[i] = g;
    sDD[i] = dD;
    sDJ[i] = dJ;
  }
  // phase A2, one thread per junction: own data + parent chain
  for (int sl = threadIdx.x; sl < nt; sl += kTopThreads) {
    const int j = ts0 + sl;
    const bool pre = sl == tid;
    const int lam = pre ? p_lam : pa.slot_lam[j];
    double yl = pre ? pre_.y : (y ? y[lam] : 0.0);
    if (upd) {
      yl -= c2 * r2[lam];
      y[lam] = yl;
    }
    if (mode == kModeDirect) yl = -yl;  // direct solve: see k_pc_up_lds
    sLam[sl] = lam;
    sY[sl] = yl;
    const int pcn = pre ? p_pcn : pa.slot_pchain[j];
    const double gp = pcn >= 0 ? 1.0 / (pre ? pre_.Tp : ldv<WT>(pa.chain_T + pcn)) : 0.0;
    sD0[sl] = gp;
    sJ0[sl] = yl + (pcn >= 0 ? (pre ? pre_.Ib : ldv<WT>(pa.chain_Ib + pcn)) : 0.0);
    const int par = pre ? p_par : pa.slot_parent[j];
    sPar[sl] = par >= 0 ? par - ts0 : -1;
    sGp[sl] = gp;
    sOff[sl] = (pre ? p_off : pa.slot_dc_off[j]) - dc0;
  }
  if (threadIdx.x == 0) sOff[nt] = ndc;
  __syncthreads();
  NX_PHASE(33);
  if constexpr (WT) NX_DSTAMP(9);
  for (int sl = threadIdx.x; sl < nt; sl += kTopThreads) {  // phase A3: fold the fixed parts
    double D0 = sD0[sl], J0 = sJ0[sl];
    for (int i = sOff[sl]; i < sOff[sl + 1]; ++i) {
      D0 += sDD[i];
      J0 += sDJ[i];
    }
    sD0[sl] = D0;
    sJ0[sl] = J0;
  }
  __syncthreads();
  NX_PHASE(34);
  // direct mode: sY holds 1 / D of every slot once its level is done (one division per
  // slot instead of two per child on the level's critical path; sY's partial is not needed)
  const bool dir = mode == kModeDirect;
  // register sweeps (top part <= kTopThreads slots with <= kWaveKids junction children
  // each -- every binary tree's): thread = slot, its level, children and their g loaded
  // into registers once, so a level costs one LDS round trip for the children's values
  // (both issued together) and the division, instead of two dependent trips per child.
  // Same arithmetic in the same order. Otherwise (a slot with more junction children): the
  // loops over LDS below.
  const int rsl = threadIdx.x;
  const bool rmine = rsl < nt;
  int rlv = -1, rnk = 0, rch[kWaveKids];
  double rg[kWaveKids];
#pragma unroll
  for (int k = 0; k < kWaveKids; ++k) {
    rch[k] = 0;
    rg[k] = 0.0;
  }
  const bool hs = pa.top_sub != nullptr;  // (uniform) wave subtrees + upper levels
  const bool hw = hs || pa.top_wave != nullptr;  // (uniform) the host's set-up, loaded up front
  if (rmine && hs && pre_.w[0] >= 0) {  // a subtree member: its wave sweeps it (rlv = -1)
  } else if (rmine && hw) {
    rlv = pre_.w[0] & 0xff;
    rnk = (pre_.w[0] >> 8) & 0xff;
#pragma unroll
    for (int k = 0; k < kWaveKids; ++k)
      if (k < rnk) {
        rch[k] = pre_.w[1 + k] & 0xfff;
        rg[k] = sG[pre_.w[1 + k] >> 12];
      }
  } else if (rmine) {
    for (int q = 0; q < nl; ++q)
      if (ts0 + rsl >= sLv[q] && ts0 + rsl < sLv[q + 1]) rlv = q;
    for (int i = sOff[rsl]; i < sOff[rsl + 1]; ++i) {
      const int chd = sChild[i];
      if (chd < 0) continue;
#pragma unroll
      for (int k = 0; k < kWaveKids; ++k)
        if (k == rnk) {
          rch[k] = chd;
          rg[k] = sG[i];
        }
      ++rnk;
    }
  }
  const bool reg = hw || (pa.top_reg && nt <= kTopThreads &&
                          __syncthreads_or(rnk > kWaveKids) == 0);
  double rD = rmine ? sD0[rsl] : 1.0, rJ = rmine ? sJ0[rsl] : 0.0, riv = 1.0;
  // wave subtrees (hs): lane = the subtree's slot (BFS order), the children's values by
  // shuffles, deepest level first -- the same arithmetic in the same order as the level
  // sweeps below; D, J (and 1 / D) of every member to LDS for the upper levels and the
  // back-substitution
  const int lsl = pre_.ls;
  const int lvl_l = (pre_.lw[0] >> 6) & 0xff, nk_l = (pre_.lw[0] >> 14) & 0xf;
  if (hs && pre_.ldep > 0) {
    int cl[kWaveKids];
    double cg[kWaveKids];
#pragma unroll
    for (int k = 0; k < kWaveKids; ++k) {
      cl[k] = k < nk_l ? pre_.lw[1 + k] & 63 : (int)(threadIdx.x & 63);
      cg[k] = k < nk_l ? sG[pre_.lw[1 + k] >> 12] : 0.0;
    }
    int kmax = nk_l;
    for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o));
    double D = lsl >= 0 ? sD0[lsl] : 1.0, J = lsl >= 0 ? sJ0[lsl] : 0.0, iv = 1.0;
    for (int q = pre_.ldep - 1; q >= 0; --q) {
#pragma unroll
      for (int k = 0; k < kWaveKids; ++k) {
        if (k >= kmax) break;
        const double Jc = __shfl(J, cl[k]);
        const double Vc = __shfl(dir ? iv : D, cl[k]);
        if (lvl_l == q && k < nk_l) {
          const double g = cg[k];
          if (dir) {
            D += g * (1.0 - g * Vc);
            J += g * Jc * Vc;
          } else {
            D += g * (1.0 - g / Vc);
            J += g * Jc / Vc;
          }
        }
      }
      if (dir && lvl_l == q) iv = 1.0 / D;
    }
    if (lsl >= 0) {
      sD[lsl] = D;
      sJ[lsl] = J;
      if (dir) sY[lsl] = iv;
    }
  }
  if (hs) __syncthreads();
  const int nlr = hs ? pa.top_sub_nup : nl;  // the levels swept block-wide
  if (reg) {
    for (int lv = nlr - 1; lv >= 0; --lv) {
      if (rlv == lv) {
        double cv[kWaveKids], cj[kWaveKids];
#pragma unroll
        for (int k = 0; k < kWaveKids; ++k) {
          cv[k] = k < rnk ? (dir ? sY[rch[k]] : sD[rch[k]]) : 1.0;
          cj[k] = k < rnk ? sJ[rch[k]] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < kWaveKids; ++k) {
          if (k >= rnk) break;
          const double g = rg[k];
          if (dir) {
            rD += g * (1.0 - g * cv[k]);
            rJ += g * cj[k] * cv[k];
          } else {
            rD += g * (1.0 - g / cv[k]);
            rJ += g * cj[k] / cv[k];
          }
        }
        if (dir) {
          riv = 1.0 / rD;
          sY[rsl] = riv;
        }
        sD[rsl] = rD;
        sJ[rsl] = rJ;
      }
      __syncthreads();
      if constexpr (WT) {
        if (lv < 16) NX_DSTAMP(12 + lv);
      }
    }
  } else
  for (int lv = nl - 1; lv >= 0; --lv) {
    for (int j = sLv[lv] + threadIdx.x; j < sLv[lv + 1]; j += kTopThreads) {
      const int sl = j - ts0;
      double D = sD0[sl], J = sJ0[sl];
      if (dir) {
        for (int i = sOff[sl]; i < sOff[sl + 1]; ++i) {
          const int ch = sChild[i];
          if (ch < 0) continue;
          const double g = sG[i], iv = sY[ch];
          D += g * (1.0 - g * iv);
          J += g * sJ[ch] * iv;
        }
        sY[sl] = 1.0 / D;
      } else {
        for (int i = sOff[sl]; i < sOff[sl + 1]; ++i) {
          const int ch = sChild[i];
          if (ch < 0) continue;
          const double g = sG[i], Dc = sD[ch];
          D += g * (1.0 - g / Dc);
          J += g * sJ[ch] / Dc;
        }
      }
      sD[sl] = D;
      sJ[sl] = J;
    }
    __syncthreads();
  }
  NX_PHASE(35);
  if constexpr (WT) NX_DSTAMP(10);
  if (MULTI && pa.n_coarse > 0) {  // back-substitution after the exchange (k_pc_coarse)
    for (int sl = threadIdx.x; sl < nt; sl += kTopThreads) {
      pa.slot_D[ts0 + sl] = sD[sl];
      pa.slot_J[ts0 + sl] = sJ[sl];
    }
    pc_coarse_partials<kTopThreads, WT>(pa, ts0, nt, sD, sJ);
    return;
  }
  double part = 0.0;
  if (reg) {  // thread = slot: z_j = (J_j + g_par z_par) / D_j, root level first
    const int p = rmine ? sPar[rsl] : -1;
    const double gp = rmine ? sGp[rsl] : 0.0;
    const int lam = rmine ? sLam[rsl] : 0;
    for (int lv = 0; lv < nlr; ++lv) {
      if (rlv == lv) {
        const double num = rJ + (p >= 0 ? gp * sJ0[p] : 0.0);
        const double zj = dir ? num * riv : num / rD;
        sJ0[rsl] = zj;  // reuse: z of top slots
        if (!dir) part += sY[rsl] * zj;
      }
      __syncthreads();
    }
    if (hs && pre_.ldep > 0) {  // the wave subtrees, root first (a subtree root's parent is
                                // an upper slot, its value in LDS)
      const int plane = (pre_.lw[0] >> 18) & 63;
      const int pq = lsl >= 0 ? sPar[lsl] : -1;
      const double gq = lsl >= 0 ? sGp[lsl] : 0.0;
      const double Jq = lsl >= 0 ? sJ[lsl] : 0.0;
      const double Vq = lsl >= 0 ? (dir ? sY[lsl] : sD[lsl]) : 1.0;
      double zq = 0.0;
      for (int q = 0; q < pre_.ldep; ++q) {
        const double zp = __shfl(zq, plane);
        if (lvl_l == q && lsl >= 0) {
          const double zpar = q == 0 ? (pq >= 0 ? sJ0[pq] : 0.0) : zp;
          const double num = Jq + (pq >= 0 ? gq * zpar : 0.0);
          zq = dir ? num * Vq : num / Vq;
        }
      }
      if (lsl >= 0) sJ0[lsl] = zq;
    }
    if (hs) {
      __syncthreads();
      if (!dir && rmine && rlv < 0) part += sY[rsl] * sJ0[rsl];  // (members: after their wave)
    }
    if constexpr (WT) NX_DSTAMP(11);
    // the stores after the levels, not inside their barriers (a workgroup barrier waits for
    // the workgroup's outstanding stores: a write-through store per level cost ~1 us each);
    // down: workgroup 0's copy only
    if (rmine && !down) {
      const double zj = sJ0[rsl];
      if (dir && pa.accum)
        z[lam] += zj;
      else
        z[lam] = zj;
      stv<WT>(pa.slot_z + ts0 + rsl, zj);
    }
    if (down && blockIdx.x == 0 && rmine) {
      pa.slot_z[ts0 + rsl] = sJ0[rsl];
      if (!pa.fres) {  // (an auxiliary solve: no publish step writes x's top values)
        if (dir && pa.accum) z[lam] += sJ0[rsl];
        else z[lam] = sJ0[rsl];
      }
    }
  } else
  for (int lv = 0; lv < nl; ++lv) {  // root level first: z_j = (J_j + g_par z_par) / D_j
    for (int j = sLv[lv] + threadIdx.x; j < sLv[lv + 1]; j += kTopThreads) {
      const int sl = j - ts0;
      const int p = sPar[sl];
      const double num = sJ[sl] + (p >= 0 ? sGp[sl] * sJ0[p] : 0.0);
      const double zj = dir ? num * sY[sl] : num / sD[sl];
      sJ0[sl] = zj;  // reuse: z of top slots
      if (!dir) part += sY[sl] * zj;
    }
    __syncthreads();
  }
  if (!reg)  // (the stores after the levels, as above)
    for (int sl = threadIdx.x; sl < nt; sl += kTopThreads) {
      const double zj = sJ0[sl];
      if (!down) {
        if (dir && pa.accum)
          z[sLam[sl]] += zj;
        else
          z[sLam[sl]] = zj;
      }
      if (!down || blockIdx.x == 0) stv<WT>(pa.slot_z + ts0 + sl, zj);
      if (down && blockIdx.x == 0 && !pa.fres) {  // (as above)
        if (dir && pa.accum) z[sLam[sl]] += zj;
        else z[sLam[sl]] = zj;
      }
    }
  NX_PHASE(36);
  if (down) {
    __syncthreads();  // the top values (sJ0) for the caller's chains
    return;
  }
  for (int sl = threadIdx.x; sl < nt; sl += kTopThreads) {  // lower-job roots read these
    pa.slot_D[ts0 + sl] = sD[sl];
    pa.slot_J[ts0 + sl] = sJ[sl];
  }
  if (!dir) block_sum_store_n<kTopThreads>(part, partB + pa.n_jobs);
  NX_PHASE_END(32);
}


template <bool MULTI>
__global__ __launch_bounds__(kTopThreads) void k_pc_top_lds(PcArgs pa, double* __restrict__ y,
                                                            const double* __restrict__ r2,
                                                            double* __restrict__ z,
                                                            const MrState* __restrict__ st,
                                                            const double* __restrict__ partA,
                                                            int nA, const double* __restrict__ red,
                                                            double* __restrict__ partB, int mode) {
  __shared__ double sD0[kCapT], sJ0[kCapT], sD[kCapT], sJ[kCapT], sGp[kCapT], sY[kCapT];
  __shared__ int sPar[kCapT], sLam[kCapT];
  __shared__ int sOff[kCapT + 1];
  __shared__ int sChild[kCapTDC];
  __shared__ double sG[kCapTDC], sDD[kCapTDC], sDJ[kCapTDC];
  __shared__ int sLv[kMaxTopLvl + 1];
  TopPre pre;
  top_pre_idx(pa, pre);
  top_pre_val(pa, y, pre);
  top_body<MULTI>(pa, y, r2, z, st, partA, nA, red, partB, mode,
                  TopLds{sD0, sJ0, sD, sJ, sGp, sY, sPar, sLam, sOff, sChild, sG, sDD, sDJ, sLv},
                  false, pre);
}

template <int BS>
__device__ void pc_prep_in_block(const PcArgs& pa, bool gcols, double* sJ, double* sZ, int* sPar,
                                 double* sTp, double* sDt, int* sCid);

// The coarse forest solve of k_pc_coarse (same arithmetic, same order) inside one
// workgroup, into sZc (n_coarse <= kCapCoarseLds); sD / sJ are scratch.
__device__ __forceinline__ void pc_coarse_lds(const PcArgs& pa, double* sD, double* sJ, double* sZc) {
  // the forest's structure is staged in LDS first (two round trips): its level sweeps
  // (13 levels each way for the 8-rank depth-17 tree) then touch no global memory
  __shared__ int sCo[kCapCoarseLds + 1], sCc[kCapCoarseLds], sCp[kCapCoarseLds];
  __shared__ int sCl[kCapCoarseLds + 1];
  __shared__ double sCg[kCapCoarseLds];
  const int nC = pa.n_coarse, nl = pa.n_clvl;
  const double* __restrict__ G = pa.cbuf + 2 * nC;
  for (int i = threadIdx.x; i <= nC; i += kPcThreads) sCo[i] = pa.c_child_off[i];
  for (int i = threadIdx.x; i <= nl; i += kPcThreads) sCl[i] = pa.c_lvl_off[i];
  for (int i = threadIdx.x; i < nC; i += kPcThreads) {
    sD[i] = pa.cbuf[i];
    sJ[i] = pa.cbuf[nC + i];
    sCg[i] = G[i];
    sCp[i] = pa.c_parent[i];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < sCo[nC]; i += kPcThreads) sCc[i] = pa.c_child[i];
  __syncthreads();
  // register sweeps (thread = coarse junction, <= kWaveKids children): its level, children
  // and their g in registers, one LDS round trip per level for the children's D, J and
  // the two divisions; same arithmetic in the same order as the loops below
  const int cj = threadIdx.x;
  const bool cmine = cj < nC;
  int clv = -1, cnk = 0, cch[kWaveKids];
#pragma unroll
  for (int k = 0; k < kWaveKids; ++k) cch[k] = 0;
  if (cmine) {
    for (int q = 0; q < nl; ++q)
      if (cj >= sCl[q] && cj < sCl[q + 1]) clv = q;
    for (int i = sCo[cj]; i < sCo[cj + 1]; ++i) {
#pragma unroll
      for (int k = 0; k < kWaveKids; ++k)
        if (k == cnk) cch[k] = sCc[i];
      ++cnk;
    }
  }
  const bool creg = nC <= kPcThreads && __syncthreads_or(cnk > kWaveKids) == 0;
  if (creg && nC <= 64) {
    // one wave (lane = coarse junction; 63 for the 8-rank C4 tree): children's D, J and the
    // parent's z by shuffles, no workgroup barrier per level; same arithmetic and order
    if (threadIdx.x < 64) {
      double D = cmine ? sD[cj] : 1.0, J = cmine ? sJ[cj] : 0.0;
      const double g0 = cmine ? sCg[cj] : 0.0;
      double gk[kWaveKids];
#pragma unroll
      for (int k = 0; k < kWaveKids; ++k) gk[k] = __shfl(g0, cch[k]);
      int kmax = cnk;
      for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o));
      for (int lv = nl - 1; lv >= 0; --lv) {
        double dk[kWaveKids], jk[kWaveKids];
#pragma unroll
        for (int k = 0; k < kWaveKids; ++k) {
          dk[k] = k < kmax ? __shfl(D, cch[k]) : 1.0;
          jk[k] = k < kmax ? __shfl(J, cch[k]) : 0.0;
        }
        if (clv == lv) {
#pragma unroll
          for (int k = 0; k < kWaveKids; ++k) {
            if (k >= cnk) break;
            D -= gk[k] * gk[k] / dk[k];
            J += gk[k] * jk[k] / dk[k];
          }
        }
      }
      const int p = cmine ? sCp[cj] : -1;
      double zc = 0.0;
      for (int lv = 0; lv < nl; ++lv) {  // root level first
        const double zp = __shfl(zc, p >= 0 ? p : cj);
        if (clv == lv) zc = (J + (p >= 0 ? g0 * zp : 0.0)) / D;
      }
      if (cmine) {
        sD[cj] = D;
        sJ[cj] = J;
        sZc[cj] = zc;
      }
    }
    __syncthreads();
    return;
  }
  if (creg) {
    double D = cmine ? sD[cj] : 1.0, J = cmine ? sJ[cj] : 0.0;
    for (int lv = nl - 1; lv >= 0; --lv) {
      if (clv == lv) {
        double g[kWaveKids], dk[kWaveKids], jk[kWaveKids];
#pragma unroll
        for (int k = 0; k < kWaveKids; ++k) {
          g[k] = k < cnk ? sCg[cch[k]] : 0.0;
          dk[k] = k < cnk ? sD[cch[k]] : 1.0;
          jk[k] = k < cnk ? sJ[cch[k]] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < kWaveKids; ++k) {
          if (k >= cnk) break;
          D -= g[k] * g[k] / dk[k];
          J += g[k] * jk[k] / dk[k];
        }
        sD[cj] = D;
        sJ[cj] = J;
      }
      __syncthreads();
    }
    const int p = cmine ? sCp[cj] : -1;
    const double gp = cmine ? sCg[cj] : 0.0;
    for (int lv = 0; lv < nl; ++lv) {  // root level first
      if (clv == lv) sZc[cj] = (J + (p >= 0 ? gp * sZc[p] : 0.0)) / D;
      __syncthreads();
    }
    return;
  }
  for (int lv = nl - 1; lv >= 0; --lv) {  // deepest level first
    for (int j = sCl[lv] + threadIdx.x; j < sCl[lv + 1]; j += kPcThreads) {
      double D = sD[j], J = sJ[j];
      for (int i = sCo[j]; i < sCo[j + 1]; ++i) {
        const int k = sCc[i];
        const double g = sCg[k], Dk = sD[k];
        D -= g * g / Dk;
        J += g * sJ[k] / Dk;
      }
      sD[j] = D;
      sJ[j] = J;
    }
    __syncthreads();
  }
  for (int lv = 0; lv < nl; ++lv) {  // root level first
    for (int j = sCl[lv] + threadIdx.x; j < sCl[lv + 1]; j += kPcThreads) {
      const int p = sCp[j];
      sZc[j] = (sJ[j] + (p >= 0 ? sCg[j] * sZc[p] : 0.0)) / sD[j];
    }
    __syncthreads();
  }
}

// The same coarse forest solve with one division per junction (its 1 / D, formed when its
// level is done; the children's terms and the back-substitution multiply by it) instead of
// two per child and one per junction on the way down: the exchange step's (k_dir_xr), where
// the coarse forest's levels (17 each way at 8 ranks) sit on the critical path. Not the
// graph path's bits (that divides), the same solution to rounding.
__device__ __forceinline__ void coarse_wave_solve_rcp(const PcArgs& pa, int w0, int w1, double D,
                                                      double J, double g0, double* sZc) {
  if (threadIdx.x >= 64) return;
  const int nC = pa.n_coarse, nl = pa.n_clvl;
  const int cj = threadIdx.x;
  const bool cmine = cj < nC;
  const int clv = cmine ? (w0 & 0xff) : -1;
  const int cnk = cmine ? ((w0 >> 8) & 0xf) : 0;
  const int p = cmine ? ((w0 >> 12) & 0xff) - 1 : -1;
  int cch[kWaveKids];
#pragma unroll
  for (int k = 0; k < kWaveKids; ++k) cch[k] = k < cnk ? (w1 >> (8 * k)) & 0xff : 0;
  double gk[kWaveKids];
#pragma unroll
  for (int k = 0; k < kWaveKids; ++k) gk[k] = __shfl(g0, cch[k]);
  int kmax = cnk;
  for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o));
  double iv = 1.0;
  for (int lv = nl - 1; lv >= 0; --lv) {
    double vk[kWaveKids], jk[kWaveKids];
#pragma unroll
    for (int k = 0; k < kWaveKids; ++k) {
      vk[k] = k < kmax ? __shfl(iv, cch[k]) : 0.0;
      jk[k] = k < kmax ? __shfl(J, cch[k]) : 0.0;
    }
    if (clv == lv) {
#pragma unroll
      for (int k = 0; k < kWaveKids; ++k) {
        if (k >= cnk) break;
        D -= gk[k] * gk[k] * vk[k];
        J += gk[k] * jk[k] * vk[k];
      }
      iv = 1.0 / D;
    }
  }
  double zc = 0.0;
  for (int lv = 0; lv < nl; ++lv) {  // root level first
    const double zp = __shfl(zc, p >= 0 ? p : cj);
    if (clv == lv) zc = (J + (p >= 0 ? g0 * zp : 0.0)) * iv;
  }
  if (cmine) sZc[cj] = zc;
}

// The coarse forest (<= 64 junctions) by one wave from registers: lane = coarse junction,
// its level, parent and children from pa.c_wave, its all-reduced D, J, G passed in; the
// same arithmetic in the same order as pc_coarse_lds. Writes z into sZc (lanes < n_coarse).
__device__ __forceinline__ void coarse_wave_solve(const PcArgs& pa, int w0, int w1, double D,
                                                  double J, double g0, double* sZc) {
  if (threadIdx.x >= 64) return;
  const int nC = pa.n_coarse, nl = pa.n_clvl;
  const int cj = threadIdx.x;
  const bool cmine = cj < nC;
  const int clv = cmine ? (w0 & 0xff) : -1;
  const int cnk = cmine ? ((w0 >> 8) & 0xf) : 0;
  const int p = cmine ? ((w0 >> 12) & 0xff) - 1 : -1;
  int cch[kWaveKids];
#pragma unroll
  for (int k = 0; k < kWaveKids; ++k) cch[k] = k < cnk ? (w1 >> (8 * k)) & 0xff : 0;
  double gk[kWaveKids];
#pragma unroll
  for (int k = 0; k < kWaveKids; ++k) gk[k] = __shfl(g0, cch[k]);
  int kmax = cnk;
  for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o));
  for (int lv = nl - 1; lv >= 0; --lv) {
    double dk[kWaveKids], jk[kWaveKids];
#pragma unroll
    for (int k = 0; k < kWaveKids; ++k) {
      dk[k] = k < kmax ? __shfl(D, cch[k]) : 1.0;
      jk[k] = k < kmax ? __shfl(J, cch[k]) : 0.0;
    }
    if (clv == lv) {
#pragma unroll
      for (int k = 0; k < kWaveKids; ++k) {
        if (k >= cnk) break;
        D -= gk[k] * gk[k] / dk[k];
        J += gk[k] * jk[k] / dk[k];
      }
    }
  }
  double zc = 0.0;
  for (int lv = 0; lv < nl; ++lv) {  // root level first
    const double zp = __shfl(zc, p >= 0 ? p : cj);
    if (clv == lv) zc = (J + (p >= 0 ? g0 * zp : 0.0)) / D;
  }
  if (cmine) sZc[cj] = zc;
}

// Several ranks, direct solve (pa.coarsedown): k_pc_coarse's work in every down workgroup.
// This thread's top slot (loaded at the sweep's start, beside its chain prefetch) ...
struct CoarsePre {
  int k, par, lvo;
  double J, D, T;
  int cw0, cw1;       // pa.c_wave: this lane's coarse junction (lanes < n_coarse)
  double cD, cJ, cG;  // its all-reduced D, J and chain conductance to the parent
};

// WT: the slots' D / J and the chains' T come from this launch (k_dir_xr: written
// write-through by other workgroups or plain by this one): loads that bypass L1
template <bool WT = false>
__device__ __forceinline__ void coarse_top_pre(const PcArgs& pa, CoarsePre& p) {
  const int sl = threadIdx.x, ts0 = pa.top_ts0, nt = pa.top_nt;
  p.k = -1;
  p.par = -1;
  p.J = 0.0;
  p.D = 1.0;
  p.T = 1.0;
  p.lvo = sl <= pa.n_top_lvl ? pa.top_lvl_off[sl] : 0;
  const int nC = pa.n_coarse;
  p.cw0 = 0;
  p.cw1 = 0;
  p.cD = 1.0;
  p.cJ = 0.0;
  p.cG = 0.0;
  if (pa.c_wave && sl < nC) {
    p.cw0 = pa.c_wave[2 * sl];
    p.cw1 = pa.c_wave[2 * sl + 1];
    p.cD = pa.cbuf[sl];
    p.cJ = pa.cbuf[nC + sl];
    p.cG = pa.cbuf[2 * nC + sl];
  }
  if (sl < nt) {
    const int j = ts0 + sl;
    p.k = pa.slot_cidx[j];
    if (p.k < 0) {
      p.par = pa.slot_parent[j];
      p.J = ldv<WT>(pa.slot_J + j);
      p.D = ldv<WT>(pa.slot_D + j);
      if (p.par >= 0) p.T = ldv<WT>(pa.chain_T + pa.slot_pchain[j]);
    }
  }
}

// ... then the coarse forest from the all-reduced [D | J | G] (pc_coarse_lds, the same bits
// on every rank and workgroup) and the top part's back-substitution (k_pc_coarse's staged
// arithmetic, thread = slot) into tZ; workgroup 0 stores the values in slot_z (the
// residual's reduce kernel moves them into x after the sweep).
__device__ __forceinline__ void coarse_top_block(const PcArgs& pa, const CoarsePre& p, double* cD, double* cJ,
                                 double* cZ, double* tZ, int* tLv) {
  const int ntl = pa.n_top_lvl, ts0 = pa.top_ts0, nt = pa.top_nt;
  const int sl = threadIdx.x;
  if (sl <= ntl) tLv[sl] = p.lvo;
  if (pa.c_wave) {  // small forest: one wave straight from the prefetched registers
    coarse_wave_solve(pa, p.cw0, p.cw1, p.cD, p.cJ, p.cG, cZ);
    __syncthreads();
  } else {
    pc_coarse_lds(pa, cD, cJ, cZ);  // ends with a barrier (tLv is staged too)
  }
  int mylv = -1;
  if (sl < nt)
    for (int q = 0; q < ntl; ++q)
      if (ts0 + sl >= tLv[q] && ts0 + sl < tLv[q + 1]) mylv = q;
  const int par = p.k >= 0 ? -2 - p.k : (p.par >= 0 ? p.par - ts0 : -1);
  for (int lv = 0; lv < ntl; ++lv) {
    if (mylv == lv) {
      double zj;
      if (par <= -2) {
        zj = cZ[-2 - par];
      } else {
        double num = p.J;
        if (par >= 0) num += tZ[par] / p.T;
        zj = num / p.D;
      }
      tZ[sl] = zj;
    }
    __syncthreads();
  }
  // workgroup 0's copy for the reduce kernel, after the levels (no global store inside the
  // level loop's barriers)
  if (blockIdx.x == 0)
    for (int i = sl; i < nt; i += kPcThreads) pa.slot_z[ts0 + i] = tZ[i];
}

// The fused halo pack (k_pack_beta's work) of the one-graph multi-rank solve: the last
// workgroup of the down sweep to finish sums this rank's beta^2 partials into red[1] and
// its slot of the gathered array, and packs the halo values of z. Resets its ticket.
__device__ void pc_pack_last(const PcArgs& pa, const double* partB, const double* z) {
  __shared__ int sLast;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    sLast = atomicAdd(pa.ticket + 1, 1) == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!sLast) return;
  __threadfence();
  const double t = block_allsum<kPcThreads>(partB, pa.n_jobs + 1);
  if (threadIdx.x == 0) {
    *pa.red1 = t;
    *pa.gath_self = t;
    pa.ticket[1] = 0;
  }
  for (int i = threadIdx.x; i < pa.n_send; i += kPcThreads) pa.send_buf[i] = z[pa.send_idx[i]];
}

// DIRK: the direct solve's instantiation (mode kModeDirect only; without the MINRES paths its
// registers fit the fused residual without spills). TOPL = false: the direct solve whose top
// part (one rank) or coarse forest (several) a launch of its own solved (pa.topdown /
// pa.coarsedown off, e.g. C4's 1024 jobs on one GPU): no top-part LDS, 141 -> 20 KB, two
// workgroups per CU instead of one
template <bool MULTI, int W, int CPL, bool DIRK, bool TOPL = true>
__global__ __launch_bounds__(kPcThreads) void k_pc_down_lds(PcArgs pa, double* __restrict__ y,
                                                            const double* __restrict__ r2,
                                                            double* __restrict__ z,
                                                            const MrState* __restrict__ st,
                                                            double* __restrict__ partB, int mode_in) {
  const int mode = DIRK ? kModeDirect : mode_in;
  // one rank, direct (pa.topdown): the top part's first indices before anything else (they
  // need no per-job offsets; the scalar loads of the prologue below would hold them back)
  TopPre tpre;
  if (DIRK && TOPL && !MULTI && pa.topdown) top_pre_idx(pa, tpre);
  __shared__ double sZ[kCapS], sA[kCapS], sB[kCapS];
  __shared__ int sP[kCapS];
  constexpr int kCT = DIRK ? 1 : kCapT;  // MINRES-only arrays (dense top, start's prep)
  __shared__ double sTa[kCT];  // dense top: a_s of every top slot
  __shared__ double sNv[kCT];  // dense top: the values this job reads, by top position
  __shared__ double sGz[kCT], sGt[kCT], sGd[kCT];  // start only: G columns (prep)
  __shared__ int sGp[kCT], sGc[kCT];
  // one rank, direct (pa.topdown): the top part's solve in every workgroup (top_body)
  constexpr int kTT = DIRK && TOPL ? kCapT : 1, kTD = DIRK && TOPL && !MULTI ? kCapTDC : 1;
  __shared__ double tD0[kTT], tJ0[kTT], tD[kTT], tJ[kTT], tGp[kTT], tY[kTT];
  __shared__ int tPar[kTT], tLam[kTT], tOff[kTT + 1], tChild[kTD];
  __shared__ double tG[kTD], tDD[kTD], tDJ[kTD];
  __shared__ int tLv[DIRK && TOPL ? kMaxTopLvl + 1 : 1];
  // several ranks, direct (pa.coarsedown): the coarse forest and the top part solved here
  // (k_pc_coarse's work) in tD0 / tJ0 / tD (coarse) and tJ (top values)
  __shared__ int sLvl[kCapLvl + 1];
  __shared__ double sCz[MULTI && TOPL ? kCapCoarseLds : 1];  // fused coarse solve
  __shared__ double sQt[DIRK ? kCapC : 1], sQb[DIRK ? kCapC : 1];  // fused residual
  // linear form: P^{-1}y is formed here and combined, z = P^{-1}y - c2 z_old, y' = y - c2 r2
  const bool lin = MULTI && pa.lin && mode == 0;
  // direct solve (mode 3): y holds b, z is the solution x; the chains form the
  // cell inputs w from b again (as k_pc_up_lds did) and finish x_q = M^{-1} (b_q - K x_s)
  const bool dir = DIRK;
  const bool fres = dir && pa.fres;  // the true residual of this job's rows
  double rr = 0.0, bb = 0.0;
  NX_PHASE_START(48);
  const int job = blockIdx.x;
  double part = 0.0;
  const int lv0 = pa.job_lvl_off[job], lv1 = pa.job_lvl_off[job + 1];
  const int js0 = lv1 > lv0 ? pa.lvl_slot_off[lv0] : 0;
  const int js1 = lv1 > lv0 ? pa.lvl_slot_off[lv1] : 0;
  const int ns = js1 - js0;
  // prefetch, independent of every z (the dense top and the level sweep below hide the
  // latency): the first chain pass's lane setup and r values, this thread's junction slot
  const int c0 = pa.job_chain_off[job], c1 = pa.job_chain_off[job + 1];
  constexpr int G = kPcThreads / W;
  const int seg = threadIdx.x / W;
  // one rank, direct (pa.topdown): the top part solved here first (k_pc_top_lds's work, same
  // arithmetic), its values left in LDS (tJ0, by top position); several ranks, direct
  // (pa.coarsedown): the coarse forest and the top part's back-substitution (k_pc_coarse's
  // work; values in tJ). Before the chain prefetch: nothing of it is live across them
  // (spills otherwise).
  const bool tdir = DIRK && TOPL && !MULTI && pa.topdown;
  const bool cdir = DIRK && TOPL && MULTI && pa.coarsedown;
  const int tts0 = pa.top_ts0;
  if constexpr (DIRK && TOPL && !MULTI) {
    if (tdir) {
      top_pre_val(pa, y, tpre);
      top_body<false>(pa, y, r2, z, st, nullptr, 0, nullptr, nullptr, kModeDirect,
                      TopLds{tD0, tJ0, tD, tJ, tGp, tY, tPar, tLam, tOff, tChild, tG, tDD, tDJ, tLv},
                      true, tpre);
    }
  }
  if constexpr (DIRK && TOPL && MULTI) {
    if (cdir) {
      CoarsePre cpre;
      coarse_top_pre(pa, cpre);
      coarse_top_block(pa, cpre, tD0, tJ0, tD, tJ, tLv);
    }
  }
  ChainLane<W, CPL> ch;
  ch.setup(pa, c0 + seg, c0 + seg < c1);
  double vc[CPL], vq[CPL], vN = 0.0;
  double mo_r[CPL];  // fused residual: the cells' R h / 6
  int ch_up = -1, ch_lo = -1, flip = 0;
  auto load_lane = [&](int c, bool active) {
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      vc[t] = ch.valid[t] ? y[ch.dof_c[t]] : 0.0;
      vq[t] = ch.valid[t] ? y[ch.dof_q[t]] : 0.0;
    }
    vN = ch.has_last ? y[ch.dof_qN] : 0.0;
    ch_up = active ? pa.chain_up[c] : -1;
    ch_lo = active ? pa.chain_lo[c] : -1;
    flip = dir && active ? pa.chain_flip[c] : 0;
  };
  load_lane(c0 + seg, c0 + seg < c1);
  int p_par = -1, p_lam = 0, p_lv = -1;
  double p_A = 0.0, p_B = 0.0, p_y = 0.0;
  const bool hwave = pa.job_wave != nullptr && lv1 > lv0 && pa.job_wave[job] > 0;
  if ((int)threadIdx.x < ns) {
    const int j = js0 + threadIdx.x;
    p_par = pa.slot_parent[j];
    p_A = pa.slot_A[j];
    p_B = pa.slot_B[j];
    p_lam = pa.slot_lam[j];
    p_y = y[p_lam];
    if (hwave) p_lv = pa.slot_wave[3 * (int64_t)j] & 0xff;  // the host's level of the slot
  }
  if (mode == 0 && st->done) return;  // after the prefetch (nothing written before)
  const double c2 = lin ? pa.xalpha[0] / st->beta : 0.0;

  // dense top (iterations, single rank): the top values this job needs, z_t = G[t,:] . a
  const bool dense = (MULTI ? pa.mdense : pa.dense) && mode == 0;
  // several ranks, fused: every workgroup solves the coarse forest (k_pc_coarse's job)
  const bool cfused = MULTI && dense && pa.fused;
  if (cfused) {
    if (pa.Gc != nullptr) {  // z_c = Gc J_c, one wave per coarse value (fixed order)
      const int nC = pa.n_coarse;
      const double* __restrict__ Jc = pa.cbuf + nC;
      const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
      for (int j = wv; j < nC; j += kPcThreads / 64) {
        const double* __restrict__ g = pa.Gc + (int64_t)j * nC;
        double acc = 0.0;
        for (int i = ln; i < nC; i += 64) acc += g[i] * Jc[i];
        acc = wave_sum(acc);
        if (ln == 0) sCz[j] = acc;
      }
      __syncthreads();
    } else {
      pc_coarse_lds(pa, sGz, sGt, sCz);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      if (lin) {
        MrState* s = const_cast<MrState*>(st);
        s->alfa = pa.xalpha[0];
        s->nb += 1;
      }
      partB[pa.n_jobs] = 0.0;  // no top kernel
    }
  }
  int nneed = 0;
  if (dense) {
    const int ts0 = pa.top_lvl_off[0], nt = pa.n_top;
    for (int sl = threadIdx.x; sl < nt; sl += kPcThreads) {  // a_s from the posted inputs
      double a = 0.0;
      if (MULTI) {
        a = pa.atop[sl];  // summed once by k_pc_cpart
      } else {
        for (int i = pa.top_uoff[sl]; i < pa.top_uoff[sl + 1]; ++i) a += pa.u[i];
      }
      sTa[sl] = a;
    }
    const int n0 = pa.job_need_off[job];
    nneed = pa.job_need_off[job + 1] - n0;
    for (int sl = threadIdx.x; sl < nt; sl += kPcThreads) sNv[sl] = 0.0;  // (never read)
    __syncthreads();
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    for (int k = wv; k < nneed; k += kPcThreads / 64) {  // one wave per needed row
      const int t = pa.job_need[n0 + k];
      const double* __restrict__ g = pa.G + (int64_t)(t - ts0) * nt;
      double acc = 0.0;
      for (int sl = ln; sl < nt; sl += 64) acc += g[sl] * sTa[sl];
      acc = wave_sum(acc);
      if (ln == 0) {
        if (MULTI) {  // + the coarse root's value through the tree
          const int rc = pa.top_rootc[t - ts0];
          if (rc >= 0) acc += pa.top_w[t - ts0] * (cfused ? sCz[rc] : pa.zc[rc]);
        }
        sNv[t - ts0] = acc;
      }
    }
    __syncthreads();
    // the job's own top rows: z and their share of r'.z
    for (int i = pa.job_tslot_off[job] + threadIdx.x; i < pa.job_tslot_off[job + 1]; i += kPcThreads) {
      const int t = pa.job_tslot[i];
      double zt = sNv[t - ts0];  // own top slots are among the needed ones
      const int lam = pa.slot_lam[t];
      double yl = y[lam];
      if (lin) {  // several ranks: linear form, as for every other row of this kernel
        zt -= c2 * z[lam];
        yl -= c2 * r2[lam];
        y[lam] = yl;
      }
      z[lam] = zt;
      part += yl * zt;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) partB[pa.n_jobs] = 0.0;  // no top kernel
  }
  auto outside = [&](int t) -> double {  // value of a top slot (outside this job)
    if (tdir) return tJ0[t - tts0];
    if (cdir) return tJ[t - tts0];
    if (!dense) return pa.slot_z[t];
    return sNv[t - pa.top_ts0];  // O(1): the job may read up to kMaxNeed top values
  };
  // phase A: every slot's A, B, parent (local index, or the parent's value for the root)
  for (int sl = threadIdx.x; sl < ns; sl += kPcThreads) {
    const int j = js0 + sl;
    const bool pre = sl == (int)threadIdx.x;  // the prefetched slot
    const int p = pre ? p_par : pa.slot_parent[j];
    const bool local = p >= js0 && p < js1;
    sA[sl] = pre ? p_A : pa.slot_A[j];
    sB[sl] = pre ? p_B : pa.slot_B[j];
    sP[sl] = local ? p - js0 : -1;
    sZ[sl] = (!local && p >= 0) ? outside(p) : 0.0;  // an outside parent is a top slot
  }
  if (lv1 > lv0 && (int)threadIdx.x <= min(lv1 - lv0, kCapLvl))
    sLvl[threadIdx.x] = pa.lvl_slot_off[lv0 + threadIdx.x];
  __syncthreads();
  NX_PHASE(49);
  if (ns <= 64 && lv1 - lv0 <= kCapLvl) {  // one wave: lane = slot, parent by shuffle
    if (threadIdx.x < 64) {
      const int sl = threadIdx.x;
      const bool mine = sl < ns;
      int mylv = hwave ? p_lv : -1;
      if (!hwave)
        for (int q = 0; q < lv1 - lv0; ++q)
          if (mine && js0 + sl >= sLvl[q] && js0 + sl < sLvl[q + 1]) mylv = q;
      const double A = mine ? sA[sl] : 0.0, Bv = mine ? sB[sl] : 0.0;
      const int p = mine ? sP[sl] : -1;
      double zv = mine ? sZ[sl] : 0.0;  // an outside parent's value for the job root
      for (int q = 0; q < lv1 - lv0; ++q) {
        const double zp = __shfl(zv, p >= 0 ? p : sl);
        if (mylv == q) zv = A + Bv * zp;
      }
      if (mine) sZ[sl] = zv;
    }
    __syncthreads();
  } else
  for (int lv = lv0; lv < lv1; ++lv) {  // phase B, root level first, LDS only
    const int la = lv - lv0 <= kCapLvl ? sLvl[lv - lv0] : pa.lvl_slot_off[lv];
    const int lb = lv - lv0 < kCapLvl ? sLvl[lv - lv0 + 1] : pa.lvl_slot_off[lv + 1];
    for (int j = la + threadIdx.x; j < lb; j += kPcThreads) {
      const int sl = j - js0;
      const int p = sP[sl];
      sZ[sl] = sA[sl] + sB[sl] * (p >= 0 ? sZ[p] : sZ[sl]);
    }
    __syncthreads();
  }
  for (int sl = threadIdx.x; sl < ns; sl += kPcThreads) {
    const bool pre = sl == (int)threadIdx.x;
    const int lam = pre ? p_lam : pa.slot_lam[js0 + sl];
    double zl = sZ[sl], yl = pre ? p_y : y[lam];
    if (lin) {
      zl -= c2 * z[lam];
      yl -= c2 * r2[lam];
      y[lam] = yl;
    }
    if (dir && pa.accum)
      z[lam] += zl;
    else
      z[lam] = zl;
    part += yl * zl;
  }
  NX_PHASE(50);
  if (fres && pa.accum) __syncthreads();  // the refined junction values above, for the check
  for (int cb = c0; cb < c1; cb += G) {
    const int c = cb + seg;
    const bool active = c < c1;
    if (cb != c0) {  // more chains than one pass: set up and load here
      ch.setup(pa, c, active);
      load_lane(c, active);
    }
    if (fres) chain_cell_mo<W, CPL>(pa, ch, c, active, flip, mo_r);
    const int up = ch_up, lo = ch_lo;
    double zt = up < 0 ? 0.0 : (up >= js0 && up < js1) ? sZ[up - js0] : outside(up);
    double zb = lo < 0 ? 0.0 : (lo >= js0 && lo < js1) ? sZ[lo - js0] : outside(lo);
    const double T = ch.T, iT = 1.0 / T;
    double rc[CPL], a[CPL], b[CPL], rq[CPL], zc[CPL];
    double sa = 0.0, sb = 0.0;
    double bcv[CPL];  // direct: b at the cells (the conservative flux recovery reads it)
    if (dir) {
#pragma unroll
      for (int t = 0; t < CPL; ++t) bcv[t] = vc[t];
      double ytop, ybot;
      direct_cell_inputs<W, CPL>(pa, ch, flip, vq, vN, vc, ytop, ybot);
    }
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      rc[t] = vc[t];
      a[t] = (T - ch.D[t]) * rc[t];
      b[t] = ch.D[t] * rc[t];
      sa += a[t];
      sb += b[t];
    }
    const double ia = seg_incl_scan<W>(sa), ib = seg_incl_scan<W>(sb);
    const double Atot = seg_sum<W>(sa);
    double pa_ = ia - sa, pb_ = ib - sb;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      pa_ += a[t];
      const double suffix = Atot - pa_ + a[t];
      const double prefix = pb_;
      pb_ += b[t];
      rq[t] = 0.0;
      zc[t] = 0.0;
      if (!ch.valid[t]) continue;
      const double Dk = ch.D[t];
      double zk = zt * (T - Dk) * iT + zb * Dk * iT + Dk * iT * suffix + (T - Dk) * iT * prefix;
      if (pa.exact) zk -= ch.mo * rc[t];  // P^{-1} of the consistent-mass Schur complement
      zc[t] = zk;
      double rk = rc[t];
      if (lin) {
        zk -= c2 * z[ch.dof_c[t]];
        rk -= c2 * r2[ch.dof_c[t]];
        y[ch.dof_c[t]] = rk;
      }
      if (dir && pa.accum)
        z[ch.dof_c[t]] += zk;
      else
        z[ch.dof_c[t]] = zk;
      part += rk * zk;
      // flux: P^{-1} r' = P^{-1} y - c2 P^{-1} r2 and z_old = P^{-1} r2, so the block is
      // applied to r' directly (z_q needs no separate linear-form correction)
      double r = vq[t];
      if (lin) {
        r -= c2 * r2[ch.dof_q[t]];
        y[ch.dof_q[t]] = r;
      }
      rq[t] = r;
    }
    double rqN = 0.0;
    if (ch.has_last) {
      rqN = vN;
      if (lin) {
        rqN -= c2 * r2[ch.dof_qN];
        y[ch.dof_qN] = rqN;
      }
    }
    if (dir) {  // x_q = M^{-1} (b_q - K x_s), conservatively (direct_flux_cons)
      double xv[CPL + 1];
      direct_flux_cons<W, CPL>(ch, flip, bcv, rq, rqN, zt, zb, xv);
#pragma unroll
      for (int t = 0; t <= CPL; ++t) {
        const bool on = t < CPL ? ch.valid[t] : ch.has_last;
        if (!on) continue;
        const int d = t < CPL ? ch.dof_q[t] : ch.dof_qN;
        if (pa.accum)
          z[d] += xv[t];
        else
          z[d] = xv[t];
      }
      if (fres) {
        if (pa.accum) {  // refinement pass: the true residual of the refined x, b - A (x + d)
#pragma unroll
          for (int t = 0; t < CPL; ++t)
            if (ch.valid[t]) {
              bcv[t] = pa.rhs_b[ch.dof_c[t]];
              rq[t] = pa.rhs_b[ch.dof_q[t]];
              zc[t] = z[ch.dof_c[t]];
              xv[t] = z[ch.dof_q[t]];
            }
          if (ch.has_last) {
            rqN = pa.rhs_b[ch.dof_qN];
            xv[CPL] = z[ch.dof_qN];
          }
          // (topdown: the top slots' x is refined by k_dir_publish_fr after this sweep, so
          // their refined value is formed here as x + d, the same single addition)
          const bool tv = tdir || cdir;  // the top values are not in x yet
          zt = up < 0 ? 0.0 : z[pa.slot_lam[up]] + (tv && (up < js0 || up >= js1) ? zt : 0.0);
          zb = lo < 0 ? 0.0 : z[pa.slot_lam[lo]] + (tv && (lo < js0 || lo >= js1) ? zb : 0.0);
        }
        direct_residual<W, CPL>(pa, ch, active, flip, bcv, rq, rqN, zc, xv, zt, zb, mo_r, rr, bb,
                                sQt, sQb, c - c0);
      }
    } else {
      part += pc_flux_block<W, CPL>(pa, ch, rq, rqN, z);
    }
  }
  NX_PHASE(51);
  if (fres) {  // multiplier rows of the junctions whose chains are all in this job
    __syncthreads();
    if ((int)threadIdx.x < ns) {
      const int j = js0 + threadIdx.x;
      if (pa.slot_rloc[j]) {
        const int pc = pa.slot_pchain[j];
        double acc = pc >= 0 ? sQb[pc - c0] : 0.0;
        for (int i = pa.slot_dc_off[j]; i < pa.slot_dc_off[j + 1]; ++i) acc += sQt[pa.slot_dc[i] - c0];
        const double bl = pa.accum ? pa.rhs_b[p_lam] : p_y;
        const double rl = bl - acc;
        pa.rres[p_lam] = rl;
        rr += rl * rl;
        bb += bl * bl;
      }
    }
    block_sum_store_n<kPcThreads>(rr, pa.rpart + job);
    __syncthreads();
    block_sum_store_n<kPcThreads>(bb, pa.rpart + pa.n_jobs + job);
  }
  if (!dir) block_sum_store_n<kPcThreads>(part, partB + blockIdx.x);
  NX_PHASE_END(48);
  if (MULTI && cfused && pa.fuse_pack) pc_pack_last(pa, partB, z);
  // single rank, start application: D is final -> factored coefficients and G here, so the
  // iterations need no separate k_pc_factor / k_pc_gbuild launches (sTa is free in mode 1)
  if (mode == 1 && (!MULTI || pa.fused)) {
    __syncthreads();
    pc_prep_in_block<kPcThreads>(pa, MULTI ? pa.mdense != 0 : pa.dense != 0, sTa, sGz, sGp, sGt,
                                 sGd, sGc);
  }
}

// ======================================================================================
// k_dir_step: the whole direct step of ONE rank in ONE launch (default; DESIGN.md section
// 3c). It replaces the four launches k_assemble_seg -> k_pc_up_lds (mode 3) ->
// k_pc_down_lds<.., true> (top part in every workgroup) -> k_dir_publish_fr. One workgroup
// per job (n_jobs <= the CU count, so all are resident; the host checks):
//   phase 1  every workgroup assembles its chains' edges -- CSR values, rhs, lumped mass,
//            k_assemble's arithmetic bit for bit -- and a strided share of the multiplier
//            rows, then runs the up sweep on the rhs it holds in registers (no reload); the
//            top part's inputs (chains at top junctions, job roots) go out write-through;
//   top      the workgroup arriving last (one agent-scope atomic each) solves the top part
//            ONCE (top_body, write-through in and out) and raises a flag; the others wait
//            for it (bounded: a workgroup that waits too long counts an error and leaves; the
//            host then resets the counters and runs the four-launch path);
//   phase 2  the down sweep from the job's own phase-1 data (same workgroup: no hand-off)
//            and the top values: x, the fused true residual (not stored: a refinement step
//            recomputes r), its partial sums and the flux-end shares of the rows no job forms
//            written through; the last workgroup to arrive sums them in a fixed order and
//            publishes the state (system-scope write-through, no L2 write-back).
// b on the multiplier rows is zero (the assembly writes zeros there; assembly.py: L[lambda]
// = 0), so no workgroup reads rhs rows another one wrote.
// ======================================================================================
// One rank's mailbox of the device-side exchange between ranks (k_dir_xr / k_dir_xg): P
// slots of each exchange's doubles (exchange 1: the coarse partials [D | J | G]; exchange
// 2: [||r||^2, ||b||^2, the cut rows' shares]), each slot ending in the launch tag of its
// writer; 2P arrival flags, one per sender; then P abort words, one per sender (64-bit:
// the reasons and the tag of the launch that gave up; an exchange fails at once on an abort
// of its own launch).
// Each rank writes its slot in every rank's mailbox (system-scope write-through stores: peer
// memory over xGMI, IPC-mapped; the in-process group: the same device), raises its flag
// there, polls its own P flags and sums the P slots in rank order.
struct XPeer {
  double* mb1;
  double* mb2;
  unsigned* fl;
};
// why an exchange step gave up (DirStep::sync[5], read by the host after the launch)
constexpr unsigned kXrFail1 = 1u;       // exchange 1 (the coarse partials) incomplete
constexpr unsigned kXrFail2 = 2u;       // exchange 2 (the residual) incomplete: x is final
constexpr unsigned kXrFailAbort = 4u;   // another rank's abort word was seen
constexpr unsigned kXrFailTag = 8u;     // a slot carried another launch's tag
constexpr unsigned kXrFailLocal = 16u;  // a workgroup of this rank gave up its local wait
constexpr unsigned kXrTopFailed = 0xffffffffu;  // sync[2]: the top part's solver gave up

struct DirStep {
  const double* edge_x;
  const double* edge_R;
  const double* edge_bc;
  const double* edge_f;  // per-edge source, or null: f everywhere
  double f;
  const int* edge_lm;
  const int* edge_seg;
  double* val;
  double* rhs;
  double* dq;
  int64_t nnz_lm, B;
  const double* lm_val;
  double* val_lm;
  double* rhs_lm;
  double* x;
  // the multiplier rows no job forms (left rows): the flux-end shares the jobs post
  const int* chain_post;  // 2 per chain: post slot of its top / bottom end, -1
  const int* left_off;    // n_left + 1: post range of every left row
  int n_left;
  double* post;
  // hand-offs: [0] phase-1 arrivals, [1] phase-2 arrivals, [2] top flag, [3] wait errors,
  // [4] the top solver's job (tagged with the launch) for its helpers
  unsigned* sync;
  unsigned epoch;  // launches since the counters were zero
  unsigned polls;  // s_sleep-paced polls before a waiting workgroup gives up (kDirWaitPolls)
  // the published state
  double rtol;
  int seq_next;
  int* seq;
  MrState* mirror;
  double* bbst;
  // k_dir_step (round 4): per job a kJobHdr-int header, per chain its edge's inputs in chain
  // order (crec: 10 doubles, ci: 4 ints) and the dynamic LDS split after the stash (doubles:
  // the phases' shared area, the top values)
  const int* job_hdr;
  const double* crec;
  const int* ci;
  int lds_main, lds_top;
  // several ranks (k_dir_xr / k_dir_xg): the ranks' mailboxes (xpeers[q]: where this rank
  // writes for rank q), this rank's own (xself: where it reads), the exchange's shape, the
  // launch tag (monotonic, never reset), the cut rows (the last xK post ranges of left_off)
  const XPeer* xpeers;
  XPeer xself;
  int xP, xrank, xld1, xld2, xK;
  unsigned xtag;
  unsigned xpoll[2];  // each exchange's poll bound (kDirWaitPolls; nx_debug_xr_polls: tests)
  int ledger;         // debug build: store classes the step drops (NX_LEDGER)
  // phase 2 by superposition (dir_sup_*; NXHIP_DIR_SUP, default 1): bit 0 on, bit 2 the
  // chain records' and lane masses' LDS copies (when they fit)
  int sup;
};

constexpr int kDirWaitPolls = 1 << 20;  // s_sleep-paced polls before a waiting workgroup gives up
// LDS of k_dir_step (doubles): the largest of phase 1, the top part and phase 2, then the
// top values (kept from the hand-off into phase 2)
constexpr int kDirLdsPhase1 = 3 * kCapC + 5 * kCapS + kCapDC + (kCapDC + kCapS + 1 + kCapLvl + 1 + 1) / 2 + 1;
constexpr int kDirLdsTop = 6 * kCapT + 3 * kCapTDC + (2 * kCapT + kCapT + 1 + kCapTDC + kMaxTopLvl + 1 + 1) / 2 + 1;
constexpr int kDirLdsPhase2 = 3 * kCapS + 2 * kCapC + (kCapS + kCapLvl + 1 + 1) / 2 + 1;
constexpr int kDirLdsMain = kDirLdsTop > kDirLdsPhase1 ? (kDirLdsTop > kDirLdsPhase2 ? kDirLdsTop : kDirLdsPhase2)
                                                       : (kDirLdsPhase1 > kDirLdsPhase2 ? kDirLdsPhase1 : kDirLdsPhase2);
constexpr int kDirLds = kDirLdsMain + kCapT;

// One chain's lane as k_dir_step assembles it (phase 1) and keeps it for phase 2 when the
// job's chains fit one pass: the cell tensors R h / 3, R h / 6 (CSR values and lumped mass;
// mo is also the residual's cell mass), the assembled b (cells, fluxes, q_N) and where the
// edge's values go. The chain lane state is rebuilt from it (dir_lane_chain: integer math,
// sums and scans) rather than kept: kept, it overflows the 128-VGPR budget of 1024 threads.
template <int W, int CPL>
struct DirLane {
  double bc[CPL], bq[CPL], bN;
  double mo[CPL];  // R h / 6; R h / 3 = 2 mo exactly (md: halving is exact in binary)
  int flip, e, sg0, seglen, s;
  __device__ __forceinline__ double md(int t) const { return 2.0 * mo[t]; }
};

// The chain lane state (ChainLane::setup without the loads) from a DirLane: the lumped flux
// mass of chain flux k (between chain cells k - 1 and k) in k_assemble's order of additions
// (so ch.rho has dq's bits) -- edge flux q: d = md_q + mo_q, then (mo_{q-1} + md_{q-1}) + d;
// q = N: mo_{N-1} + md_{N-1}.
template <int W, int CPL>
__device__ __forceinline__ void dir_lane_chain(const PcArgs& pa, const DirLane<W, CPL>& L,
                                               bool active, ChainLane<W, CPL>& ch) {
#pragma clang fp contract(off)
  const int N = pa.N;
  const int l = lane_of<W>();
  const int flip = L.flip;
  const int64_t base = (int64_t)L.e * (2 * N + 1);
  double md[CPL];
#pragma unroll
  for (int t = 0; t < CPL; ++t) md[t] = L.md(t);
  const double* mo = L.mo;
  const double mdP = __shfl_up(md[CPL - 1], 1, W), moP = __shfl_up(mo[CPL - 1], 1, W);
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    const int k = l * CPL + t;
    ch.valid[t] = active && k < N;
    const int kp = flip ? N - 1 - k : k;
    const int qp = flip ? N - k : k;
    ch.dof_c[t] = (int)(base + 2 * kp + 1);
    ch.dof_q[t] = (int)(base + 2 * qp);
    ch.rho[t] = 0.0;
    if (!ch.valid[t]) continue;
    const double mdq = t > 0 ? md[t - 1] : mdP, moq = t > 0 ? mo[t - 1] : moP;  // cell k - 1
    double d;
    if (!flip) {  // edge flux k: cells k - 1 and k
      d = md[t] + mo[t];
      if (k > 0) d = (moq + mdq) + d;
    } else if (k > 0) {  // edge flux N - k: edge cells N - k (chain k - 1) and N - k - 1 (chain k)
      d = mdq + moq;
      d = (mo[t] + md[t]) + d;
    } else {  // edge flux N: edge cell N - 1 (chain cell 0) only
      d = mo[t] + md[t];
    }
    ch.rho[t] = d;
  }
  // chain flux N (the lane holding chain cell N - 1): edge flux N (its last cell) or, flipped,
  // edge flux 0 (its first cell)
  ch.has_last = active && (l == (N - 1) / CPL);
  ch.dof_qN = (int)(base + 2 * (flip ? 0 : N));
  ch.rhoN = 0.0;
  {
    const int tl = (N - 1) - l * CPL;
    double mdl = 0.0, mol = 0.0;
#pragma unroll
    for (int t = 0; t < CPL; ++t)
      if (t == tl) {
        mdl = md[t];
        mol = mo[t];
      }
    if (ch.has_last) ch.rhoN = flip ? mdl + mol : mol + mdl;
  }
  // ChainLane::setup's mo: the edge's q_0 lumped mass / 3 (chain flux 0, or N when flipped)
  const double dq0 = flip ? __shfl(ch.rhoN, (N - 1) / CPL, W) : __shfl(ch.rho[0], 0, W);
  ch.mo = active ? dq0 / 3.0 : 1.0;
  ch.finish();
}

// One chain's edge assembled in registers by its W lanes (lane = CPL cells, chain order):
// cell tensors R h / 3, R h / 6 and the rhs as k_assemble computes them. Nothing is stored
// here (dir_chain_store).
template <int W, int CPL>
__device__ __forceinline__ void dir_chain_asm(const PcArgs& pa, const DirStep& da, int c,
                                              bool active, DirLane<W, CPL>& L) {
#pragma clang fp contract(off)
  const int N = pa.N;
  const int l = threadIdx.x & (W - 1);
  const int e = active ? pa.chain_edge[c] : 0;
  const int flip = active ? pa.chain_flip[c] : 0;
  L.e = e;
  L.flip = flip;
  double x0[3], x1[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    x0[i] = da.edge_x[6 * (int64_t)e + i];
    x1[i] = da.edge_x[6 * (int64_t)e + 3 + i];
  }
  const double R = da.edge_R[e];
  const double fe = da.edge_f ? da.edge_f[e] : da.f;
  const double bc0 = da.edge_bc[2 * (int64_t)e], bc1 = da.edge_bc[2 * (int64_t)e + 1];
  L.s = da.edge_lm[2 * (int64_t)e] >= 0;
  L.sg0 = da.edge_seg[e];
  L.seglen = da.edge_seg[e + 1] - L.sg0;
  const double invN = pa.invN;
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    const int k = l * CPL + t;
    const bool valid = active && k < N;
    const int kp = flip ? N - 1 - k : k;
    const int qp = flip ? N - k : k;
    L.mo[t] = 0.0;
    L.bc[t] = 0.0;
    L.bq[t] = 0.0;
    if (valid) {
      double va[3], vb[3];
      vertex(x0, x1, kp, N, invN, va);
      vertex(x0, x1, kp + 1, N, invN, vb);
      const double d0 = vb[0] - va[0], d1 = vb[1] - va[1], d2 = vb[2] - va[2];
      const double h = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
      L.mo[t] = R * h / 6.0;  // (R h / 3 = 2 L.mo[t], bit for bit)
      L.bc[t] = -(fe * h);  // negated pressure row: -(f h)
      L.bq[t] = qp == 0 ? bc0 : (qp == N ? bc1 : 0.0);
    }
  }
  L.bN = (active && l == (N - 1) / CPL) ? (flip ? bc0 : bc1) : 0.0;
}

// The assembly's stores of one chain's edge from its lane state: rhs, lumped mass, and the
// CSR segment (entry i by lane i mod W, unit stride; the tensors of the entry's cells fetched
// by shuffles; uniform trip count across the wave -- the longest segment, 7N + 3 -- so every
// shuffle has all lanes).
// UNIT: the CSR segment in k_assemble's order instead (entry i by lane i mod W, unit stride
// over the lanes: whole cache lines per store; the tensors of the entry's cells fetched by
// shuffles, ~2x the issue time) -- the workgroups that store while waiting for the top part,
// where the issue time is hidden and partially written lines would cost HBM traffic.
template <int W, int CPL, bool UNIT = false>
__device__ __forceinline__ void dir_chain_store(const PcArgs& pa, const DirStep& da, bool active,
                                                const DirLane<W, CPL>& L) {
  ChainLane<W, CPL> ch;
  dir_lane_chain<W, CPL>(pa, L, active, ch);
  const int N = pa.N;
  const int l = threadIdx.x & (W - 1);
  const int flip = L.flip;
  const int64_t qb = (int64_t)L.e * (N + 1);
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    if (!ch.valid[t]) continue;
    const int k = l * CPL + t;
    if (!NX_LEDGER(da, 2)) {
      da.rhs[ch.dof_c[t]] = L.bc[t];
      da.rhs[ch.dof_q[t]] = L.bq[t];
    }
    if (da.dq) da.dq[qb + (flip ? N - k : k)] = ch.rho[t];
  }
  if (ch.has_last) {
    if (!NX_LEDGER(da, 2)) da.rhs[ch.dof_qN] = L.bN;
    if (da.dq) da.dq[qb + (flip ? 0 : N)] = ch.rhoN;
  }
  if (NX_LEDGER(da, 1)) return;
  // the CSR segment, each lane its own cells' rows (edge order: cell g owns p_g's 2 entries
  // and q_{g+1}'s 5 -- q_N's 3 + s_dst for g = N - 1 -- from q0len + 7 g on; cell 0 also the
  // q_0 row): values as decode_entry lists them, the next edge cell's masses from the
  // neighbouring lane (chain cell k + 1, or k - 1 on a flipped chain)
  if constexpr (UNIT) {
    const int smax = 7 * N + 3;
    for (int ib = 0; ib < smax; ib += W) {
      const int i = ib + l;
      const bool in = active && i < L.seglen;
      const Entry en = decode_entry(in ? i : 0, N, L.s);
      const int ca = en.cell, cb = min(en.cell + 1, N - 1);
      const int ka = flip ? N - 1 - ca : ca, kb = flip ? N - 1 - cb : cb;
      double mdA = 0.0, moA = 0.0, mdB = 0.0;
#pragma unroll
      for (int t = 0; t < CPL; ++t) {
        const double b = __shfl(L.mo[t], ka / CPL, W), a = 2.0 * b;
        const double m2 = 2.0 * __shfl(L.mo[t], kb / CPL, W);
        if (ka % CPL == t) {
          mdA = a;
          moA = b;
        }
        if (kb % CPL == t) mdB = m2;
      }
      double v;
      switch (en.vk) {
        case V_P1: v = 1.0; break;
        case V_M1: v = -1.0; break;
        case V_MD: v = mdA; break;
        case V_MO: v = moA; break;
        default: v = mdA + mdB; break;  // interior diagonal: cells g and g+1
      }
      if (in) da.val[L.sg0 + i] = v;
    }
    return;
  }
  const int s0 = L.s, q0len = 3 + s0;
  const int sdst = L.seglen - (7 * N + 1 + s0);
  const double moD = __shfl_down(L.mo[0], 1, W), mdD = 2.0 * moD;
  const double moU = __shfl_up(L.mo[CPL - 1], 1, W), mdU = 2.0 * moU;
  double* __restrict__ v = da.val + L.sg0;
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    if (!ch.valid[t]) continue;
    const int k = l * CPL + t;
    const int g = flip ? N - 1 - k : k;
    const double md = L.md(t), mo = L.mo[t];
    double* o = v + q0len + 7 * g;
    o[0] = 1.0;
    o[1] = -1.0;
    o[2] = mo;
    o[3] = -1.0;
    if (g < N - 1) {  // the next edge cell: chain cell k + 1 (k - 1 when flipped)
      double mdn, mon;
      if (!flip) {
        mdn = t + 1 < CPL ? L.md(t + 1) : mdD;
        mon = t + 1 < CPL ? L.mo[t + 1] : moD;
      } else {
        mdn = t > 0 ? L.md(t - 1) : mdU;
        mon = t > 0 ? L.mo[t - 1] : moU;
      }
      o[4] = md + mdn;
      o[5] = 1.0;
      o[6] = mon;
    } else {
      o[4] = md;
      if (sdst) o[5] = 1.0;
    }
    if (g == 0) {  // row q_0: [q_0, p_0, q_1, (lambda_src)]
      v[0] = md;
      v[1] = 1.0;
      v[2] = mo;
      if (s0) v[3] = -1.0;
    }
  }
}

// Phase 1: assembly + up sweep (k_pc_up_lds's mode-3 arithmetic; b_lambda = 0).
// keep (the job's chains fit one pass): the assembly's stores are left to the caller
// (dir_chain_store after the hand-off) and the lane state stays in L for phase 2; the slot's
// back-substitution coefficients (thread = slot) are returned in sA_ / sB_ either way.
// MULTI (k_dir_team_up): every chain's T / It / Ib and every slot's D / J / A / B also go to
// global memory (the separate down sweep after the coarse all-reduce reads them), as
// k_pc_up_lds stores them.
// store_now: the assembly's stores in the pass loop (k_dir_team_up with several chain
// passes); otherwise they come after the hand-off (dir_stores_all).
template <int W, int CPL, bool MULTI = false>
__device__ __forceinline__ void dir_up_fused(const PcArgs& pa, const DirStep& da,
                                             double* lds, DirLane<W, CPL>& L, bool store_now,
                                             double& sA_, double& sB_) {
  double* sT = lds;
  double* sIt = sT + kCapC;
  double* sIb = sIt + kCapC;
  double* sD0 = sIb + kCapC;
  double* sJ0 = sD0 + kCapS;
  double* sD = sJ0 + kCapS;
  double* sJ = sD + kCapS;
  double* sIv = sJ + kCapS;
  double* sG = sIv + kCapS;
  int* sChild = reinterpret_cast<int*>(sG + kCapDC);
  int* sOff = sChild + kCapDC;
  int* sLvl = sOff + kCapS + 1;
  const int job = blockIdx.x;
  const int c0 = pa.job_chain_off[job], c1 = pa.job_chain_off[job + 1];
  constexpr int G = kPcThreads / W;
  const int seg = threadIdx.x / W, l = threadIdx.x & (W - 1);
  const int ts0 = pa.top_ts0, ts1 = pa.top_ts0 + pa.top_nt;
  const int lv0 = pa.job_lvl_off[job], lv1 = pa.job_lvl_off[job + 1];
  const int js0 = lv1 > lv0 ? pa.lvl_slot_off[lv0] : 0;
  const int js1 = lv1 > lv0 ? pa.lvl_slot_off[lv1] : 0;
  // prefetch of this thread's junction slot of phase A (independent of the chains)
  constexpr int kPre = 4;
  int p_pcn = -1, p_o0 = 0, p_o1 = 0, p_dc[kPre], p_lo[kPre];
  if ((int)threadIdx.x < js1 - js0) {
    const int j = js0 + threadIdx.x;
    p_pcn = pa.slot_pchain[j];
    p_o0 = pa.slot_dc_off[j];
    p_o1 = pa.slot_dc_off[j + 1];
#pragma unroll
    for (int q = 0; q < kPre; ++q) {
      const bool in = p_o0 + q < p_o1;
      p_dc[q] = in ? pa.slot_dc[p_o0 + q] : 0;
      p_lo[q] = in ? pa.dc_lo[p_o0 + q] : -1;
    }
  }
  for (int cb = c0; cb < c1; cb += G) {
    const int c = cb + seg;
    const bool active = c < c1;
    const int cu = active ? pa.chain_up[c] : -1, clo = active ? pa.chain_lo[c] : -1;
    dir_chain_asm<W, CPL>(pa, da, c, active, L);
    if (store_now) dir_chain_store<W, CPL>(pa, da, active, L);
    ChainLane<W, CPL> ch;
    dir_lane_chain<W, CPL>(pa, L, active, ch);
    double vc[CPL];
#pragma unroll
    for (int t = 0; t < CPL; ++t) vc[t] = L.bc[t];
    double ytop = 0.0, ybot = 0.0;
    direct_cell_inputs<W, CPL>(pa, ch, L.flip, L.bq, L.bN, vc, ytop, ybot);
    double sr = 0.0, srd = 0.0;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      if (!ch.valid[t]) continue;
      sr += vc[t];
      srd += vc[t] * ch.D[t];
    }
    sr = seg_sum<W>(sr);
    srd = seg_sum<W>(srd);
    if (active && l == 0) {
      const double ib = srd / ch.T;
      const double it = (sr - ib) + ytop, ibe = ib + ybot;  // + the multiplier rows' share
      sT[c - c0] = ch.T;
      sIb[c - c0] = ibe;
      sIt[c - c0] = it;
      if ((cu >= ts0 && cu < ts1) || (clo >= ts0 && clo < ts1)) {  // the top part reads it
        st_wt(pa.chain_T + c, ch.T);
        st_wt(pa.chain_It + c, it);
        st_wt(pa.chain_Ib + c, ibe);
      } else if (MULTI) {
        pa.chain_T[c] = ch.T;
        pa.chain_It[c] = it;
        pa.chain_Ib[c] = ibe;
      }
    }
  }
  NX_DSTAMP(32);
  if (lv1 <= lv0) return;
  const int jwave = pa.job_wave ? pa.job_wave[job] : 0;
  int wv0 = 0, wv1 = 0, wv2 = 0;
  if (jwave > 0 && (int)threadIdx.x < js1 - js0) {
    const int* w = pa.slot_wave + 3 * (int64_t)(js0 + threadIdx.x);
    wv0 = w[0];
    wv1 = w[1];
    wv2 = w[2];
  }
  const int ns = js1 - js0;
  const int dc0 = pa.slot_dc_off[js0];
  __syncthreads();
  for (int sl = threadIdx.x; sl < ns; sl += kPcThreads) {  // phase A
    const int j = js0 + sl;
    const bool pre = sl == (int)threadIdx.x;
    const int pcn = pre ? p_pcn : pa.slot_pchain[j];
    double D0 = pcn >= 0 ? 1.0 / sT[pcn - c0] : 0.0;
    double J0 = pcn >= 0 ? sIb[pcn - c0] : 0.0;  // (- b_lambda = -0 added: no change)
    const int o0 = pre ? p_o0 : pa.slot_dc_off[j], o1 = pre ? p_o1 : pa.slot_dc_off[j + 1];
    sOff[sl] = o0 - dc0;
    for (int i = o0; i < o1; ++i) {
      const int q = i - o0;
      const bool pq = pre && q < kPre;
      int dcq = 0, loq = -1;
#pragma unroll
      for (int r = 0; r < kPre; ++r)
        if (r == q) {
          dcq = p_dc[r];
          loq = p_lo[r];
        }
      const int cl = (pq ? dcq : pa.slot_dc[i]) - c0;
      const int lo = pq ? loq : pa.dc_lo[i];
      const double g = 1.0 / sT[cl];
      J0 += sIt[cl];
      if (lo >= 0) {
        sChild[i - dc0] = lo - js0;
        sG[i - dc0] = g;
      } else {
        sChild[i - dc0] = -1;
        D0 += g;
      }
    }
    sD0[sl] = D0;
    sJ0[sl] = J0;
  }
  if (threadIdx.x == 0) sOff[ns] = pa.slot_dc_off[js1] - dc0;
  if ((int)threadIdx.x <= min(lv1 - lv0, kCapLvl)) sLvl[threadIdx.x] = pa.lvl_slot_off[lv0 + threadIdx.x];
  __syncthreads();
  NX_DSTAMP(33);
  bool wave_lv = jwave > 0;
  if (!wave_lv) {
    int nkids = 0;
    if ((int)threadIdx.x < ns)
      for (int i = sOff[threadIdx.x]; i < sOff[threadIdx.x + 1]; ++i) nkids += sChild[i] >= 0;
    wave_lv = __syncthreads_or(nkids > kWaveKids) == 0 && ns <= 64 && lv1 - lv0 <= kCapLvl;
  }
  if (wave_lv) {  // one wave: lane = slot, the children's values by shuffles
    if (threadIdx.x < 64) {
      const int sl = threadIdx.x;
      const bool mine = sl < ns;
      int mylv = -1;
      int cl[kWaveKids];
      double cg[kWaveKids];
#pragma unroll
      for (int k = 0; k < kWaveKids; ++k) {
        cl[k] = sl;
        cg[k] = 0.0;
      }
      int nk = 0, kmax;
      if (jwave > 0) {
        kmax = jwave - 1;
        if (mine) {
          mylv = wv0 & 0xff;
          nk = (wv0 >> 8) & 0xff;
          const int cw[kWaveKids] = {wv1 & 0xffff, wv1 >> 16, wv2 & 0xffff, wv2 >> 16};
#pragma unroll
          for (int k = 0; k < kWaveKids; ++k)
            if (k < nk) {
              cl[k] = cw[k] & 63;
              cg[k] = sG[cw[k] >> 6];
            }
        }
      } else {
        for (int q = 0; q < lv1 - lv0; ++q)
          if (mine && js0 + sl >= sLvl[q] && js0 + sl < sLvl[q + 1]) mylv = q;
        if (mine)
          for (int i = sOff[sl]; i < sOff[sl + 1]; ++i) {
            const int chd = sChild[i];
            if (chd < 0) continue;
#pragma unroll
            for (int k = 0; k < kWaveKids; ++k)
              if (k == nk) {
                cl[k] = chd;
                cg[k] = sG[i];
              }
            ++nk;
          }
        kmax = nk;
        for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o));
      }
      double D = mine ? sD0[sl] : 1.0, J = mine ? sJ0[sl] : 0.0, iv = 1.0;
      for (int q = lv1 - lv0 - 1; q >= 0; --q) {
#pragma unroll
        for (int k = 0; k < kWaveKids; ++k) {
          if (k >= kmax) break;
          const double Jc = __shfl(J, cl[k]);
          const double Dc = __shfl(iv, cl[k]);
          if (mylv == q && k < nk) {
            const double g = cg[k];
            D += g * (1.0 - g * Dc);
            J += g * Jc * Dc;
          }
        }
        if (mylv == q) iv = 1.0 / D;
      }
      if (mine) {
        sD[sl] = D;
        sJ[sl] = J;
        sIv[sl] = iv;
      }
    }
    __syncthreads();
  } else {
    for (int lv = lv1 - 1; lv >= lv0; --lv) {  // deepest level first
      const int la = lv - lv0 <= kCapLvl ? sLvl[lv - lv0] : pa.lvl_slot_off[lv];
      const int lb = lv - lv0 < kCapLvl ? sLvl[lv - lv0 + 1] : pa.lvl_slot_off[lv + 1];
      for (int j = la + threadIdx.x; j < lb; j += kPcThreads) {
        const int sl = j - js0;
        double D = sD0[sl], J = sJ0[sl];
        for (int i = sOff[sl]; i < sOff[sl + 1]; ++i) {
          const int ch = sChild[i];
          if (ch < 0) continue;
          const double g = sG[i], iv = sIv[ch];
          D += g * (1.0 - g * iv);
          J += g * sJ[ch] * iv;
        }
        sIv[sl] = 1.0 / D;
        sD[sl] = D;
        sJ[sl] = J;
      }
      __syncthreads();
    }
  }
  NX_DSTAMP(34);
  // back-substitution coefficients (own phase 2 reads them); the job's root level hands its
  // (D, J) to the top part
  const int root1 = sLvl[1];
  if ((int)threadIdx.x < ns) {  // ns <= kCapS < kPcThreads: thread = slot
    const int sl = threadIdx.x;
    const int j = js0 + sl;
    const int pcn = p_pcn;
    const double J = sJ[sl], iv = sIv[sl];
    sA_ = J * iv;
    sB_ = pcn >= 0 ? iv / sT[pcn - c0] : 0.0;
    if (j < root1) {
      st_wt(pa.slot_D + j, sD[sl]);
      st_wt(pa.slot_J + j, J);
    } else if (MULTI) {
      pa.slot_D[j] = sD[sl];
      pa.slot_J[j] = J;
    }
    if (MULTI) {
      pa.slot_A[j] = sA_;
      pa.slot_B[j] = sB_;
    }
  }
}

// The state to the host-coherent mirror with system-scope write-through stores (no release
// fence: this XCD's L2, dirty with x, is not written back first), the stamp after them.
__device__ __forceinline__ void publish_wt(const MrState& s, int q, int* seq, MrState* mirror) {
  *seq = q;  // device count of published states (read by later launches)
  MrState o = s;
  o.pad = 0;
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&o);
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(mirror);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(MrState) / 8); ++i)
    __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  vm_drain();
  __hip_atomic_store(&mirror->pad, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// sum_{k0 <= k < k1} post[k] in order, write-through loads: the first four issued together
// (a left row has one post per incident chain: three on a binary tree), not one round trip
// each
__device__ __forceinline__ double post_sum(const double* post, int k0, int k1) {
  double v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = k0 + j < k1 ? ld_wt(post + k0 + j) : 0.0;
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (k0 + j < k1) acc += v[j];
  for (int k = k0 + 4; k < k1; ++k) acc += ld_wt(post + k);
  return acc;
}

// The last workgroup of phase 2: the partials and the left rows' shares, fixed order.
// lo0 / lo1: left row threadIdx.x's post range (loaded by every workgroup before its
// arrival: static), so only the write-through loads remain after the hand-off.
__device__ __forceinline__ void dir_publish_fused(const PcArgs& pa, const DirStep& da, int lo0,
                                                  int lo1) {
#pragma clang fp contract(off)
  __shared__ double s_r[kPcThreads / 64], s_b[kPcThreads / 64];
  const int nj = pa.n_jobs;
  double rr = 0.0, bb = 0.0;
  for (int i = threadIdx.x; i < nj; i += kPcThreads) {
    rr += ld_wt(pa.rpart + i);
    bb += ld_wt(pa.rpart + nj + i);
  }
  for (int i = threadIdx.x; i < da.n_left; i += kPcThreads) {
    const bool pre = i == (int)threadIdx.x;
    const int k0 = pre ? lo0 : da.left_off[i], k1 = pre ? lo1 : da.left_off[i + 1];
    const double rv = 0.0 - post_sum(da.post, k0, k1);  // b = 0 on the multiplier rows
    rr += rv * rv;
  }
  rr = wave_sum(rr);
  bb = wave_sum(bb);
  NX_DSTAMP(23);
  if ((threadIdx.x & 63) == 0) {
    s_r[threadIdx.x >> 6] = rr;
    s_b[threadIdx.x >> 6] = bb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    rr = 0.0;
    bb = 0.0;
    for (int w = 0; w < kPcThreads / 64; ++w) {
      rr += s_r[w];
      bb += s_b[w];
    }
    NX_DSTAMP(24);
    da.bbst[0] = bb;
    MrState s{};
    s.beta1 = sqrt(bb);
    s.relres = bb > 0.0 ? sqrt(rr / bb) : sqrt(rr);
    s.rtol = da.rtol;
    s.it = 1;
    s.done = 1;
    s.converged = s.relres <= da.rtol ? 1 : 0;
    publish_wt(s, da.seq_next, da.seq, da.mirror);
  }
}

// The assembly's stores of one workgroup (after its hand-off): a strided share of the
// multiplier rows (+-1 values, zero rhs), then its chains' edges -- from the kept lanes
// (keep: one chain pass) or re-assembled pass by pass.
template <int W, int CPL, bool UNIT = false>
__device__ __forceinline__ void dir_stores_all(const PcArgs& pa, const DirStep& da, int job,
                                               bool keep, DirLane<W, CPL>& L) {
  const int nj = pa.n_jobs;
  const int64_t nlm = da.nnz_lm > da.B ? da.nnz_lm : da.B;
  for (int64_t i = (int64_t)job * kPcThreads + threadIdx.x; i < nlm; i += (int64_t)nj * kPcThreads) {
    if (i < da.nnz_lm && !NX_LEDGER(da, 16)) da.val_lm[i] = da.lm_val[i];
    if (i < da.B && !NX_LEDGER(da, 16)) da.rhs_lm[i] = 0.0;
  }
  const int c0 = pa.job_chain_off[job], c1 = pa.job_chain_off[job + 1];
  if (keep) {
    dir_chain_store<W, CPL, UNIT>(pa, da, c0 + (int)threadIdx.x / W < c1, L);
    return;
  }
  constexpr int G = kPcThreads / W;
  for (int cb = c0; cb < c1; cb += G) {
    const int c = cb + (int)threadIdx.x / W;
    dir_chain_asm<W, CPL>(pa, da, c, c < c1, L);
    dir_chain_store<W, CPL, UNIT>(pa, da, c < c1, L);
  }
}

// ---- k_dir_step's job description (round 4) ------------------------------------------
// A workgroup of the fused step used to reach its first arithmetic through four dependent
// rounds of global loads (job offsets -> level offsets -> chains -> their edges) and loaded
// its static slot / chain data again after each hand-off. Now: per job a kJobHdr-int header
// (host-built: c0, c1, lv0, lv1, js0, js1, dc0, dc1, jwave, root1), per chain its edge's
// inputs in chain order (crec: x_u[3], x_v[3], R, f, b(q_0), b(q_N); ci: edge, flip | s << 1,
// CSR segment start, length; refreshed whenever the coefficients change), and every static
// array the job's phases read staged in LDS once (the stash) -- two dependent rounds (the
// header; then the stash and the chain records, issued together) before the workgroup
// computes, and none after the hand-offs except the handed-over values themselves.
constexpr int kJobHdr = 16;

struct ChainRec {
  double x0[3], x1[3], R, fe, bc0, bc1;
  int e, flip, s, sg0, seglen;
};

// The lane's chain c0 + threadIdx.x / W, formed afresh: a re-assembly late in the step then
// forms its record addresses again instead of keeping the first load's (a 64-bit address
// live through the whole step -- spilled to scratch at the 128-VGPR budget)
template <int W>
__device__ __forceinline__ int fresh_chain(int c0) {
  int c = c0 + (int)threadIdx.x / W;
  asm volatile("" : "+v"(c));
  return c;
}

__device__ __forceinline__ void chain_rec_load(const DirStep& da, int c, bool active,
                                               ChainRec& r) {
  const int cc = active ? c : 0;
  const double* p = da.crec + 10 * (int64_t)cc;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    r.x0[i] = p[i];
    r.x1[i] = p[3 + i];
  }
  r.R = p[6];
  r.fe = p[7];
  r.bc0 = p[8];
  r.bc1 = p[9];
  const int4 q = *reinterpret_cast<const int4*>(da.ci + 4 * (int64_t)cc);
  r.e = active ? q.x : 0;
  r.flip = active ? (q.y & 1) : 0;
  r.s = q.y >> 1;
  r.sg0 = q.z;
  r.seglen = q.w;
}

// A chain record in LDS (12 doubles per lane group, field i by lane i % W of the group): the
// top solver's copy of its job's records (DirStep::sup & 4)
constexpr int kRecLds = 12;
template <int W>
__device__ __forceinline__ void rec_to_lds(double* base, bool active, const ChainRec& r) {
  if (!active) return;
  const int l = threadIdx.x & (W - 1);
  double* o = base + kRecLds * (int)(threadIdx.x / W);
  const double ints0 = __builtin_bit_cast(double, (long long)(unsigned)r.e |
                                                      ((long long)(r.flip | (r.s << 1)) << 32));
  const double ints1 = __builtin_bit_cast(double, (long long)(unsigned)r.sg0 |
                                                      ((long long)r.seglen << 32));
#pragma unroll
  for (int i = 0; i < kRecLds; ++i)
    if (i % W == l) {
      const double v = i < 3 ? r.x0[i] : i < 6 ? r.x1[i - 3] : i == 6 ? r.R : i == 7 ? r.fe
                       : i == 8 ? r.bc0 : i == 9 ? r.bc1 : i == 10 ? ints0 : ints1;
      o[i] = v;
    }
}
template <int W>
__device__ __forceinline__ void rec_from_lds(const double* base, bool active, ChainRec& r) {
  const double* o = base + kRecLds * (int)(threadIdx.x / W);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    r.x0[i] = active ? o[i] : 0.0;
    r.x1[i] = active ? o[3 + i] : 0.0;
  }
  r.R = active ? o[6] : 0.0;
  r.fe = active ? o[7] : 0.0;
  r.bc0 = active ? o[8] : 0.0;
  r.bc1 = active ? o[9] : 0.0;
  const long long a = active ? __builtin_bit_cast(long long, o[10]) : 0;
  const long long b = active ? __builtin_bit_cast(long long, o[11]) : 0;
  r.e = (int)(a & 0xffffffffll);
  const int fs = (int)(a >> 32);
  r.flip = fs & 1;
  r.s = fs >> 1;
  r.sg0 = (int)(b & 0xffffffffll);
  r.seglen = (int)(b >> 32);
}

// A lane state (DirLane) from the LDS copies: the cell masses and cell rhs as phase 1
// assembled them (lpark: 2 CPL per thread), the flux rhs and the indices from the chain's
// record -- dir_chain_asm_rec's values, bit for bit, without its arithmetic
template <int W, int CPL>
__device__ __forceinline__ void lane_from_lds(const PcArgs& pa, const double* rec_lds,
                                              const double* lpark, bool active,
                                              DirLane<W, CPL>& L) {
  ChainRec r;
  rec_from_lds<W>(rec_lds, active, r);
  const int N = pa.N;
  const int l = threadIdx.x & (W - 1);
  const int flip = r.flip;
  L.e = r.e;
  L.flip = flip;
  L.s = r.s;
  L.sg0 = r.sg0;
  L.seglen = r.seglen;
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    const int k = l * CPL + t;
    const bool valid = active && k < N;
    const int qp = flip ? N - k : k;
    L.mo[t] = lpark[t * kPcThreads + threadIdx.x];
    L.bc[t] = lpark[(CPL + t) * kPcThreads + threadIdx.x];
    L.bq[t] = valid ? (qp == 0 ? r.bc0 : (qp == N ? r.bc1 : 0.0)) : 0.0;
  }
  L.bN = (active && l == (N - 1) / CPL) ? (flip ? r.bc0 : r.bc1) : 0.0;
}

// dir_chain_asm from a chain record (the same arithmetic, the same bits)
template <int W, int CPL>
__device__ __forceinline__ void dir_chain_asm_rec(const PcArgs& pa, const ChainRec& r, bool active,
                                                  DirLane<W, CPL>& L) {
#pragma clang fp contract(off)
  const int N = pa.N;
  const int l = threadIdx.x & (W - 1);
  const int flip = r.flip;
  L.e = r.e;
  L.flip = flip;
  L.s = r.s;
  L.sg0 = r.sg0;
  L.seglen = r.seglen;
  const double invN = pa.invN;
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    const int k = l * CPL + t;
    const bool valid = active && k < N;
    const int kp = flip ? N - 1 - k : k;
    const int qp = flip ? N - k : k;
    L.mo[t] = 0.0;
    L.bc[t] = 0.0;
    L.bq[t] = 0.0;
    if (valid) {
      double va[3], vb[3];
      vertex(r.x0, r.x1, kp, N, invN, va);
      vertex(r.x0, r.x1, kp + 1, N, invN, vb);
      const double d0 = vb[0] - va[0], d1 = vb[1] - va[1], d2 = vb[2] - va[2];
      const double h = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
      L.mo[t] = r.R * h / 6.0;  // (R h / 3 = 2 L.mo[t], bit for bit)
      L.bc[t] = -(r.fe * h);  // negated pressure row: -(f h)
      L.bq[t] = qp == 0 ? r.bc0 : (qp == N ? r.bc1 : 0.0);
    }
  }
  L.bN = (active && l == (N - 1) / CPL) ? (flip ? r.bc0 : r.bc1) : 0.0;
}

// The job's static arrays in LDS at the start of the dynamic LDS (ints, fixed offsets, so
// the stash costs no registers): level slot offsets (absolute slot ids), per slot its parent
// chain, parent slot, multiplier row, own-row flag (slot_rloc), one-wave set-up (3) and
// down-chain offsets (absolute), per down-chain entry its chain and lower slot, per chain of
// the first pass its end slots and post slots. The host checks the job sizes against the caps.
constexpr int kStLv = 256, kStNs = kCapS, kStNd = kCapDC, kStNc = 256;
constexpr int kOffLv = 0, kOffPc = kOffLv + kStLv, kOffPar = kOffPc + kStNs,
              kOffLam = kOffPar + kStNs, kOffRl = kOffLam + kStNs, kOffW0 = kOffRl + kStNs,
              kOffW1 = kOffW0 + kStNs, kOffW2 = kOffW1 + kStNs, kOffDco = kOffW2 + kStNs,
              kOffSdc = kOffDco + kStNs + 8, kOffDlo = kOffSdc + kStNd, kOffCup = kOffDlo + kStNd,
              kOffClo = kOffCup + kStNc, kOffCpt = kOffClo + kStNc, kOffCpb = kOffCpt + kStNc,
              kStashInts = kOffCpb + kStNc;
constexpr int kStashDbl = (kStashInts + 1) / 2;

struct JobStash {
  int c0, c1, lv0, lv1, js0, js1, dc0, dc1, jwave, root1;
  int* base;
  __device__ __forceinline__ int& lv(int i) const { return base[kOffLv + i]; }
  __device__ __forceinline__ int& pchain(int i) const { return base[kOffPc + i]; }
  __device__ __forceinline__ int& par(int i) const { return base[kOffPar + i]; }
  __device__ __forceinline__ int& lam(int i) const { return base[kOffLam + i]; }
  __device__ __forceinline__ int& rloc(int i) const { return base[kOffRl + i]; }
  __device__ __forceinline__ int& w0(int i) const { return base[kOffW0 + i]; }
  __device__ __forceinline__ int& w1(int i) const { return base[kOffW1 + i]; }
  __device__ __forceinline__ int& w2(int i) const { return base[kOffW2 + i]; }
  __device__ __forceinline__ int& dcoff(int i) const { return base[kOffDco + i]; }
  __device__ __forceinline__ int& sdc(int i) const { return base[kOffSdc + i]; }
  __device__ __forceinline__ int& dlo(int i) const { return base[kOffDlo + i]; }
  __device__ __forceinline__ int& cup(int i) const { return base[kOffCup + i]; }
  __device__ __forceinline__ int& clo(int i) const { return base[kOffClo + i]; }
  __device__ __forceinline__ int& cpt(int i) const { return base[kOffCpt + i]; }
  __device__ __forceinline__ int& cpb(int i) const { return base[kOffCpb + i]; }
};

// this thread's share of the stash, loaded (job_stash_load) before the caller issues its
// chain records, written to LDS after (job_stash_store): the loads fly together
struct StashRegs {
  int lv, pc, par, lam, rl, w0, w1, w2, off, sdc, dlo, cu, cl, pt, pb;
};

template <int W>
__device__ __forceinline__ void job_stash_load(const PcArgs& pa, const DirStep& da, int job,
                                               int* base, JobStash& S, StashRegs& R) {
  const int4* hd = reinterpret_cast<const int4*>(da.job_hdr + kJobHdr * (int64_t)job);
  const int4 h0 = hd[0], h1 = hd[1], h2 = hd[2];
  S.c0 = h0.x;
  S.c1 = h0.y;
  S.lv0 = h0.z;
  S.lv1 = h0.w;
  S.js0 = h1.x;
  S.js1 = h1.y;
  S.dc0 = h1.z;
  S.dc1 = h1.w;
  S.jwave = h2.x;
  S.root1 = h2.y;
  S.base = base;
  const int t = threadIdx.x;
  const int nlv = S.lv1 - S.lv0, ns = S.js1 - S.js0, nd = S.dc1 - S.dc0;
  const int nc = min(S.c1 - S.c0, kPcThreads / W);
  const int j = S.js0 + t, c = S.c0 + t, i = S.dc0 + t;
  const bool sl = t < ns, wv = sl && S.jwave > 0;
  R.lv = t <= nlv ? pa.lvl_slot_off[S.lv0 + t] : 0;
  R.pc = sl ? pa.slot_pchain[j] : -1;
  R.par = sl ? pa.slot_parent[j] : -1;
  R.lam = sl ? pa.slot_lam[j] : 0;
  R.rl = sl ? pa.slot_rloc[j] : 0;
  R.w0 = wv ? pa.slot_wave[3 * (int64_t)j] : 0;
  R.w1 = wv ? pa.slot_wave[3 * (int64_t)j + 1] : 0;
  R.w2 = wv ? pa.slot_wave[3 * (int64_t)j + 2] : 0;
  R.off = t <= ns ? pa.slot_dc_off[j] : 0;
  R.sdc = t < nd ? pa.slot_dc[i] : 0;
  R.dlo = t < nd ? pa.dc_lo[i] : -1;
  const bool ch = t < nc;
  R.cu = ch ? pa.chain_up[c] : -1;
  R.cl = ch ? pa.chain_lo[c] : -1;
  R.pt = ch && da.chain_post ? da.chain_post[2 * (int64_t)c] : -1;
  R.pb = ch && da.chain_post ? da.chain_post[2 * (int64_t)c + 1] : -1;
}

__device__ __forceinline__ void job_stash_store(const JobStash& S, const StashRegs& R, int nc) {
  const int t = threadIdx.x;
  const int nlv = S.lv1 - S.lv0, ns = S.js1 - S.js0, nd = S.dc1 - S.dc0;
  if (t <= nlv) S.lv(t) = R.lv;
  if (t < ns) {
    S.pchain(t) = R.pc;
    S.par(t) = R.par;
    S.lam(t) = R.lam;
    S.rloc(t) = R.rl;
    S.w0(t) = R.w0;
    S.w1(t) = R.w1;
    S.w2(t) = R.w2;
  }
  if (t <= ns) S.dcoff(t) = R.off;
  if (t < nd) {
    S.sdc(t) = R.sdc;
    S.dlo(t) = R.dlo;
  }
  if (t < nc) {
    S.cup(t) = R.cu;
    S.clo(t) = R.cl;
    S.cpt(t) = R.pt;
    S.cpb(t) = R.pb;
  }
}

// Phase 1 from the stash (dir_up_fused's arithmetic, the same bits): the chains' edges
// assembled in registers from their records (rec: the first pass's, loaded by the caller),
// the up sweep, the top part's inputs posted write-through; sA_ / sB_ the slot's
// back-substitution coefficients (thread = slot). MULTI: every chain's T / It / Ib and
// every slot's D / J / A / B also to global memory, as k_pc_up_lds stores them.
template <int W, int CPL>
__device__ __forceinline__ void dir_sup_chain_core(const ChainLane<W, CPL>& ch,
                                                   const DirLane<W, CPL>& L, const double* vc,
                                                   double* park);
// the job's slots in one wave with the host-built set-up: phase 1's junction phases then run
// in wave 0 alone (no workgroup barriers), and the superposition's chain part is split
// around them (dir_up_v2, dir_sup_core_wave0)
__device__ __forceinline__ bool sup_wslots(const JobStash& S) {
  return S.jwave > 0 && S.js1 - S.js0 <= 64 && S.lv1 > S.lv0;
}

template <int W, int CPL, bool MULTI = false>
__device__ __forceinline__ void dir_up_v2(const PcArgs& pa, const DirStep& da, double* lds,
                                          const JobStash& S, ChainRec& rec, DirLane<W, CPL>& L,
                                          double& sA_, double& sB_, double* park = nullptr) {
  double* sT = lds;
  double* sIt = sT + kCapC;
  double* sIb = sIt + kCapC;
  double* sD0 = sIb + kCapC;
  double* sJ0 = sD0 + kCapS;
  double* sD = sJ0 + kCapS;
  double* sJ = sD + kCapS;
  double* sIv = sJ + kCapS;
  double* sG = sIv + kCapS;
  int* sChild = reinterpret_cast<int*>(sG + kCapDC);
  int* sOff = sChild + kCapDC;
  const int c0 = S.c0, c1 = S.c1;
  constexpr int G = kPcThreads / W;
  const int seg = threadIdx.x / W, l = threadIdx.x & (W - 1);
  const int ts0 = pa.top_ts0, ts1 = pa.top_ts0 + pa.top_nt;
  const int lv0 = S.lv0, lv1 = S.lv1;
  const int js0 = S.js0, js1 = S.js1;
  // superposition (park, one chain pass) with the job's slots in one wave (the host-built
  // one-wave set-up): wave 0 alone runs the junction phases, with no workgroup barrier after
  // the chains' one, and the other waves run their chains' u-independent part meanwhile;
  // wave 0 runs its own after the hand-off (dir_sup_core_wave0), in the wait
  const bool wslots = park && sup_wslots(S);
  const bool core_now = park && !wslots;
  for (int cb = c0; cb < c1; cb += G) {
    const int c = cb + seg;
    const bool active = c < c1;
    if (cb != c0) chain_rec_load(da, c, active, rec);
    const int cu = !active ? -1 : (cb == c0 ? S.cup(seg) : pa.chain_up[c]);
    const int clo = !active ? -1 : (cb == c0 ? S.clo(seg) : pa.chain_lo[c]);
    dir_chain_asm_rec<W, CPL>(pa, rec, active, L);
    ChainLane<W, CPL> ch;
    dir_lane_chain<W, CPL>(pa, L, active, ch);
    double vc[CPL];
#pragma unroll
    for (int t = 0; t < CPL; ++t) vc[t] = L.bc[t];
    double ytop = 0.0, ybot = 0.0;
    direct_cell_inputs<W, CPL>(pa, ch, L.flip, L.bq, L.bN, vc, ytop, ybot);
    // phase 2's u-independent part of the chain (superposition, one pass), here while its
    // lane state is at hand -- or kept for after the barrier (wslots)
    if (core_now) {
      dir_sup_chain_core<W, CPL>(ch, L, vc, park);
    } else if (park) {  // (the cell inputs wait in the park's cell slots, not in registers)
#pragma unroll
      for (int t = 0; t < CPL; ++t) park[t * kPcThreads + threadIdx.x] = vc[t];
    }
    double sr = 0.0, srd = 0.0;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      if (!ch.valid[t]) continue;
      sr += vc[t];
      srd += vc[t] * ch.D[t];
    }
    sr = seg_sum<W>(sr);
    srd = seg_sum<W>(srd);
    if (active && l == 0) {
      const double ib = srd / ch.T;
      const double it = (sr - ib) + ytop, ibe = ib + ybot;  // + the multiplier rows' share
      sT[c - c0] = ch.T;
      sIb[c - c0] = ibe;
      sIt[c - c0] = it;
      if ((cu >= ts0 && cu < ts1) || (clo >= ts0 && clo < ts1)) {  // the top part reads it
        st_wt(pa.chain_T + c, ch.T);
        st_wt(pa.chain_It + c, it);
        st_wt(pa.chain_Ib + c, ibe);
      } else if (MULTI) {
        pa.chain_T[c] = ch.T;
        pa.chain_It[c] = it;
        pa.chain_Ib[c] = ibe;
      }
    }
  }
  NX_DSTAMP(32);
  if (lv1 <= lv0) return;
  const int jwave = S.jwave;
  const int ns = js1 - js0;
  const int dc0 = S.dc0;
  __syncthreads();
  NX_DSTAMP(33);
  if (wslots && threadIdx.x >= 64) {  // the other waves: their chains' part, then leave
    ChainLane<W, CPL> ch;
    dir_lane_chain<W, CPL>(pa, L, c0 + seg < c1, ch);
    double vc[CPL];
#pragma unroll
    for (int t = 0; t < CPL; ++t) vc[t] = park[t * kPcThreads + threadIdx.x];
    dir_sup_chain_core<W, CPL>(ch, L, vc, park);
    return;
  }
  for (int sl = threadIdx.x; sl < ns; sl += kPcThreads) {  // phase A (ns <= kCapS: one pass)
    const int pcn = S.pchain(sl);
    double D0 = pcn >= 0 ? 1.0 / sT[pcn - c0] : 0.0;
    double J0 = pcn >= 0 ? sIb[pcn - c0] : 0.0;  // (- b_lambda = -0 added: no change)
    const int o0 = S.dcoff(sl), o1 = S.dcoff(sl + 1);
    sOff[sl] = o0 - dc0;
    for (int i = o0; i < o1; ++i) {
      const int cl = S.sdc(i - dc0) - c0;
      const int lo = S.dlo(i - dc0);
      const double g = 1.0 / sT[cl];
      J0 += sIt[cl];
      if (lo >= 0) {
        sChild[i - dc0] = lo - js0;
        sG[i - dc0] = g;
      } else {
        sChild[i - dc0] = -1;
        D0 += g;
      }
    }
    sD0[sl] = D0;
    sJ0[sl] = J0;
  }
  if (threadIdx.x == 0) sOff[ns] = S.dc1 - dc0;
  if (wslots) {
    wave_lds_sync();
  } else {
    __syncthreads();
  }
  bool wave_lv = jwave > 0;
  if (!wave_lv) {
    int nkids = 0;
    if ((int)threadIdx.x < ns)
      for (int i = sOff[threadIdx.x]; i < sOff[threadIdx.x + 1]; ++i) nkids += sChild[i] >= 0;
    wave_lv = __syncthreads_or(nkids > kWaveKids) == 0 && ns <= 64 && lv1 - lv0 <= kCapLvl;
  }
  if (wave_lv) {  // one wave: lane = slot, the children's values by shuffles
    if (threadIdx.x < 64) {
      const int sl = threadIdx.x;
      const bool mine = sl < ns;
      int mylv = -1;
      int cl[kWaveKids];
      double cg[kWaveKids];
#pragma unroll
      for (int k = 0; k < kWaveKids; ++k) {
        cl[k] = sl;
        cg[k] = 0.0;
      }
      int nk = 0, kmax;
      if (jwave > 0) {
        kmax = jwave - 1;
        if (mine) {
          const int wv0 = S.w0(sl), wv1 = S.w1(sl), wv2 = S.w2(sl);
          mylv = wv0 & 0xff;
          nk = (wv0 >> 8) & 0xff;
          const int cw[kWaveKids] = {wv1 & 0xffff, wv1 >> 16, wv2 & 0xffff, wv2 >> 16};
#pragma unroll
          for (int k = 0; k < kWaveKids; ++k)
            if (k < nk) {
              cl[k] = cw[k] & 63;
              cg[k] = sG[cw[k] >> 6];
            }
        }
      } else {
        for (int q = 0; q < lv1 - lv0; ++q)
          if (mine && js0 + sl >= S.lv(q) && js0 + sl < S.lv(q + 1)) mylv = q;
        if (mine)
          for (int i = sOff[sl]; i < sOff[sl + 1]; ++i) {
            const int chd = sChild[i];
            if (chd < 0) continue;
#pragma unroll
            for (int k = 0; k < kWaveKids; ++k)
              if (k == nk) {
                cl[k] = chd;
                cg[k] = sG[i];
              }
            ++nk;
          }
        kmax = nk;
        for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o));
      }
      double D = mine ? sD0[sl] : 1.0, J = mine ? sJ0[sl] : 0.0, iv = 1.0;
      for (int q = lv1 - lv0 - 1; q >= 0; --q) {
#pragma unroll
        for (int k = 0; k < kWaveKids; ++k) {
          if (k >= kmax) break;
          const double Jc = __shfl(J, cl[k]);
          const double Dc = __shfl(iv, cl[k]);
          if (mylv == q && k < nk) {
            const double g = cg[k];
            D += g * (1.0 - g * Dc);
            J += g * Jc * Dc;
          }
        }
        if (mylv == q) iv = 1.0 / D;
      }
      if (mine) {
        sD[sl] = D;
        sJ[sl] = J;
        sIv[sl] = iv;
      }
    }
    if (wslots) {
      wave_lds_sync();
    } else {
      __syncthreads();
    }
  } else {
    for (int lv = lv1 - 1; lv >= lv0; --lv) {  // deepest level first
      const int la = S.lv(lv - lv0), lb = S.lv(lv - lv0 + 1);
      for (int j = la + threadIdx.x; j < lb; j += kPcThreads) {
        const int sl = j - js0;
        double D = sD0[sl], J = sJ0[sl];
        for (int i = sOff[sl]; i < sOff[sl + 1]; ++i) {
          const int ch = sChild[i];
          if (ch < 0) continue;
          const double g = sG[i], iv = sIv[ch];
          D += g * (1.0 - g * iv);
          J += g * sJ[ch] * iv;
        }
        sIv[sl] = 1.0 / D;
        sD[sl] = D;
        sJ[sl] = J;
      }
      __syncthreads();
    }
  }
  NX_DSTAMP(34);
  // back-substitution coefficients (own phase 2 reads them); the job's root level hands its
  // (D, J) to the top part
  const int root1 = S.root1;
  if ((int)threadIdx.x < ns) {  // ns <= kCapS < kPcThreads: thread = slot
    const int sl = threadIdx.x;
    const int j = js0 + sl;
    const int pcn = S.pchain(sl);
    const double J = sJ[sl], iv = sIv[sl];
    sA_ = J * iv;
    sB_ = pcn >= 0 ? iv / sT[pcn - c0] : 0.0;
    if (j < root1) {
      st_wt(pa.slot_D + j, sD[sl]);
      st_wt(pa.slot_J + j, J);
    } else if (MULTI) {
      pa.slot_D[j] = sD[sl];
      pa.slot_J[j] = J;
    }
    if (MULTI) {
      pa.slot_A[j] = sA_;
      pa.slot_B[j] = sB_;
    }
  }
}

// Phase 2 from the stash (k_pc_down_lds's mode-3 arithmetic with the fused residual, r not
// stored): sTop the top part's values by top position; keep: the job's chains in one pass,
// their lane state still in L from phase 1; sA_ / sB_: this thread's slot coefficients.
template <int W, int CPL>
__device__ __forceinline__ void dir_down_v2(const PcArgs& pa, const DirStep& da, double* lds,
                                            const double* sTop, const JobStash& S,
                                            const DirLane<W, CPL>& L, bool keep, double sA_,
                                            double sB_, int job) {
  // (contraction as in k_pc_down_lds: the same x bit for bit)
  double* sZ = lds;
  double* sA = sZ + kCapS;
  double* sB = sA + kCapS;
  double* sQt = sB + kCapS;
  double* sQb = sQt + kCapC;
  int* sP = reinterpret_cast<int*>(sQb + kCapC);
  __shared__ double s_w[2 * (kPcThreads / 64)];
  // (job: this rank's job index -- the in-process group's launch holds every rank's jobs)
  const int ts0 = pa.top_ts0;
  const int lv0 = S.lv0, lv1 = S.lv1;
  const int js0 = S.js0, js1 = S.js1;
  const int ns = js1 - js0;
  const int c0 = S.c0, c1 = S.c1;
  constexpr int G = kPcThreads / W;
  const int seg = threadIdx.x / W, l = threadIdx.x & (W - 1);
  double* __restrict__ x = da.x;
  const double* __restrict__ b = da.rhs;  // this job's own rows (written by this workgroup)
  ChainLane<W, CPL> ch;
  double vc[CPL], vq[CPL], vN = 0.0, mo_r[CPL];
  int ch_up = -1, ch_lo = -1, flip = 0, post_t = -1, post_b = -1;
  auto load_lane = [&](int c, bool active) {
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      vc[t] = ch.valid[t] ? b[ch.dof_c[t]] : 0.0;
      vq[t] = ch.valid[t] ? b[ch.dof_q[t]] : 0.0;
    }
    vN = ch.has_last ? b[ch.dof_qN] : 0.0;
    ch_up = active ? pa.chain_up[c] : -1;
    ch_lo = active ? pa.chain_lo[c] : -1;
    flip = active ? pa.chain_flip[c] : 0;
    post_t = active ? da.chain_post[2 * (int64_t)c] : -1;
    post_b = active ? da.chain_post[2 * (int64_t)c + 1] : -1;
  };
  if (keep) {  // phase 1's lane; the chain's ends and posts from the stash
    const bool active = c0 + seg < c1;
    dir_lane_chain<W, CPL>(pa, L, active, ch);
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      vc[t] = L.bc[t];
      vq[t] = L.bq[t];
      mo_r[t] = L.mo[t];
    }
    vN = L.bN;
    ch_up = active ? S.cup(seg) : -1;
    ch_lo = active ? S.clo(seg) : -1;
    flip = L.flip;
    post_t = active ? S.cpt(seg) : -1;
    post_b = active ? S.cpb(seg) : -1;
  } else {
    ch.setup(pa, c0 + seg, c0 + seg < c1);
    load_lane(c0 + seg, c0 + seg < c1);
  }
  const bool hwave = S.jwave > 0 && lv1 > lv0;
  // phase A: every slot's A, B, parent (local index, or the parent's value: a top slot)
  if ((int)threadIdx.x < ns) {  // (ns <= kCapS < kPcThreads: thread = slot)
    const int sl = threadIdx.x;
    const int p = S.par(sl);
    const bool local = p >= js0 && p < js1;
    sA[sl] = sA_;
    sB[sl] = sB_;
    sP[sl] = local ? p - js0 : -1;
    sZ[sl] = (!local && p >= 0) ? sTop[p - ts0] : 0.0;
  }
  __syncthreads();
  NX_DSTAMP(36);
  if (ns <= 64 && lv1 - lv0 <= kCapLvl) {  // one wave: lane = slot, parent by shuffle
    if (threadIdx.x < 64) {
      const int sl = threadIdx.x;
      const bool mine = sl < ns;
      int mylv = hwave && mine ? S.w0(sl) & 0xff : -1;
      if (!hwave)
        for (int q = 0; q < lv1 - lv0; ++q)
          if (mine && js0 + sl >= S.lv(q) && js0 + sl < S.lv(q + 1)) mylv = q;
      const double A = mine ? sA[sl] : 0.0, Bv = mine ? sB[sl] : 0.0;
      const int p = mine ? sP[sl] : -1;
      double zv = mine ? sZ[sl] : 0.0;
      for (int q = 0; q < lv1 - lv0; ++q) {
        const double zp = __shfl(zv, p >= 0 ? p : sl);
        if (mylv == q) zv = A + Bv * zp;
      }
      if (mine) sZ[sl] = zv;
    }
    __syncthreads();
  } else {
    for (int lv = lv0; lv < lv1; ++lv) {  // root level first
      const int la = S.lv(lv - lv0), lb = S.lv(lv - lv0 + 1);
      for (int j = la + threadIdx.x; j < lb; j += kPcThreads) {
        const int sl = j - js0;
        const int p = sP[sl];
        sZ[sl] = sA[sl] + sB[sl] * (p >= 0 ? sZ[p] : sZ[sl]);
      }
      __syncthreads();
    }
  }
  NX_DSTAMP(37);
  if ((int)threadIdx.x < ns && !NX_LEDGER(da, 4)) x[S.lam(threadIdx.x)] = sZ[threadIdx.x];
  double rr = 0.0, bb = 0.0;
  for (int cb = c0; cb < c1; cb += G) {
    const int c = cb + seg;
    const bool active = c < c1;
    if (cb != c0) {  // more chains than one pass: set up and load here
      ch.setup(pa, c, active);
      load_lane(c, active);
    }
    if (!keep) chain_cell_mo<W, CPL>(pa, ch, c, active, flip, mo_r);
    const int up = ch_up, lo = ch_lo;
    const double zt = up < 0 ? 0.0 : (up >= js0 && up < js1) ? sZ[up - js0] : sTop[up - ts0];
    const double zb = lo < 0 ? 0.0 : (lo >= js0 && lo < js1) ? sZ[lo - js0] : sTop[lo - ts0];
    const double T = ch.T, iT = 1.0 / T;
    double bcv[CPL], a[CPL], bs[CPL], zc[CPL];
#pragma unroll
    for (int t = 0; t < CPL; ++t) bcv[t] = vc[t];
    {
      double ytop, ybot;
      direct_cell_inputs<W, CPL>(pa, ch, flip, vq, vN, vc, ytop, ybot);
    }
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      a[t] = (T - ch.D[t]) * vc[t];
      bs[t] = ch.D[t] * vc[t];
      sa += a[t];
      sb += bs[t];
    }
    const double ia = seg_incl_scan<W>(sa), ibv = seg_incl_scan<W>(sb);
    const double Atot = seg_sum<W>(sa);
    double pa_ = ia - sa, pb_ = ibv - sb;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      pa_ += a[t];
      const double suffix = Atot - pa_ + a[t];
      const double prefix = pb_;
      pb_ += bs[t];
      zc[t] = 0.0;
      if (!ch.valid[t]) continue;
      const double Dk = ch.D[t];
      double zk = zt * (T - Dk) * iT + zb * Dk * iT + Dk * iT * suffix + (T - Dk) * iT * prefix;
      zk -= ch.mo * vc[t];  // the consistent-mass Schur complement
      zc[t] = zk;
      if (!NX_LEDGER(da, 4)) x[ch.dof_c[t]] = zk;
    }
    double xv[CPL + 1];
    direct_flux_cons<W, CPL>(ch, flip, bcv, vq, vN, zt, zb, xv);
#pragma unroll
    for (int t = 0; t <= CPL; ++t) {
      const bool on = t < CPL ? ch.valid[t] : ch.has_last;
      if (on && !NX_LEDGER(da, 4)) x[t < CPL ? ch.dof_q[t] : ch.dof_qN] = xv[t];
    }
    direct_residual<W, CPL, false>(pa, ch, active, flip, bcv, vq, vN, zc, xv, zt, zb, mo_r, rr, bb,
                                   sQt, sQb, c - c0);
    // the chain's ends at rows no job forms: their flux shares, write-through
    if (active && l == 0 && post_t >= 0) st_wt(da.post + post_t, sQt[c - c0]);
    if (ch.has_last && post_b >= 0) st_wt(da.post + post_b, sQb[c - c0]);
  }
  __syncthreads();
  NX_DSTAMP(38);
  // multiplier rows of the junctions whose chains are all in this job (b_lambda = 0)
  if ((int)threadIdx.x < ns && S.rloc(threadIdx.x)) {
    const int sl = threadIdx.x;
    const int pc = S.pchain(sl);
    double acc = pc >= 0 ? sQb[pc - c0] : 0.0;
    for (int i = S.dcoff(sl); i < S.dcoff(sl + 1); ++i) acc += sQt[S.sdc(i - S.dc0) - c0];
    const double rl = 0.0 - acc;
    rr += rl * rl;
  }
  rr = wave_sum(rr);
  bb = wave_sum(bb);
  if ((threadIdx.x & 63) == 0) {
    s_w[threadIdx.x >> 6] = rr;
    s_w[kPcThreads / 64 + (threadIdx.x >> 6)] = bb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tr = s_w[0], tb = s_w[kPcThreads / 64];
    for (int i = 1; i < kPcThreads / 64; ++i) {
      tr += s_w[i];
      tb += s_w[kPcThreads / 64 + i];
    }
    st_wt(pa.rpart + job, tr);
    st_wt(pa.rpart + pa.n_jobs + job, tb);
  }
}

// ---- phase 2 by superposition (round 6; DirStep::sup) --------------------------------------
// A job's down sweep is affine in the few top values it reads: a root slot's value is
// A + B u (u = its parent's top value), a lower slot's A + B z_parent, and a chain's cells
// and fluxes are affine in its end values (zt, zb): the cells
//   z_k = zt (T - D_k) / T + zb D_k / T + [D_k suffix_k + (T - D_k) prefix_k] / T - mo w_k,
// the fluxes x_q[k] = q_0 - s P_k with T q_0 = s1 + s s2 - s (zb - zt) (direct_flux_cons).
// So everything that does not depend on u -- the chain lane state, the Thomas scans of
// M^{-1} b_q, the prefix sums, every slot's particular value z_p (u = 0) and its response
// H = dz / du with the top value it hangs from (rho) -- runs BEFORE the top values arrive:
// the chains' part in phase 1 on its lane state (dir_sup_chain_core; the Thomas scans are
// phase 1's own), the slots' part in the wait (dir_sup_slots). After them only
// z = z_p + H u per slot, z_k += zt (T - D_k) / T + zb D_k / T, x_q += s (zt - zb) / T, the
// fused true residual from those final values (registers and shuffles; no loads) and the
// partial sums remain (dir_sup_finish). x itself is stored after the phase-2 hand-off
// (dir_sup_store_x): nothing of this launch reads it, and its drain then stays off the
// hand-off. Same solution in exact arithmetic; the additions are ordered differently, so x
// differs from the launches' x by rounding (tests: 1e-14), and the residual reported is
// that of the stored x, bit for bit.
// LDS: the slots' arrays in their own region after the top values (sup: sA, sB, sZp, sH,
// kCapS doubles each; ints sRho, sP) -- the top part's solver fills them during its own
// wait, so they must survive the top part -- then the lanes' park; sQt, sQb [kCapC] in the
// phases' shared area (smem).
constexpr int kDirLdsSupSlots = 5 * kCapS;

__device__ __forceinline__ bool sup_one_wave(const JobStash& S) {
  return S.js1 - S.js0 <= 64 && S.lv1 - S.lv0 <= kCapLvl;
}

// Every slot's particular value z_p, its response H and the top position rho it hangs from
// (-1: none), in the slots' region sup (A, B: phase 1's coefficients, kCapS each, then z_p,
// H, rho).
// One wave when the job's slots fit (no block barrier: the caller's next barrier publishes
// them), else level sweeps in LDS (every thread must call).
template <int W, int CPL>
__device__ __forceinline__ void dir_sup_slots(const PcArgs& pa, double* sup, const JobStash& S) {
  const bool slt = (int)threadIdx.x < kCapS;
  double* sA = sup;
  double* sB = sA + kCapS;
  double* sZp = sB + kCapS;
  double* sH = sZp + kCapS;
  int* sRho = reinterpret_cast<int*>(sH + kCapS);
  int* sP = sRho + kCapS;
  const double sA_ = slt ? sA[threadIdx.x] : 0.0, sB_ = slt ? sB[threadIdx.x] : 0.0;
  const int ts0 = pa.top_ts0;
  const int lv0 = S.lv0, lv1 = S.lv1, js0 = S.js0, js1 = S.js1;
  const int ns = js1 - js0;
  if (sup_one_wave(S)) {
    if (threadIdx.x < 64) {  // lane = slot, the parent's (z_p, H, rho) by shuffles
      const int sl = threadIdx.x;
      const bool mine = sl < ns;
      const bool hwave = S.jwave > 0 && lv1 > lv0;
      int mylv = hwave && mine ? S.w0(sl) & 0xff : -1;
      if (!hwave)
        for (int q = 0; q < lv1 - lv0; ++q)
          if (mine && js0 + sl >= S.lv(q) && js0 + sl < S.lv(q + 1)) mylv = q;
      const int p = mine ? S.par(sl) : -1;
      const bool local = p >= js0 && p < js1;
      const int pl = local ? p - js0 : sl;
      double zv = sA_, hv = (mine && !local && p >= 0) ? sB_ : 0.0;
      int rho = (mine && !local && p >= 0) ? p - ts0 : -1;
      for (int q = 1; q < lv1 - lv0; ++q) {  // (level 0: the roots, set above)
        const double zp = __shfl(zv, pl), hp = __shfl(hv, pl);
        const int rp = __shfl(rho, pl);
        if (mylv == q && local) {
          zv = sA_ + sB_ * zp;
          hv = sB_ * hp;
          rho = rp;
        }
      }
      if (mine) {
        sZp[sl] = zv;
        sH[sl] = hv;
        sRho[sl] = rho;
      }
    }
    return;
  }
  if ((int)threadIdx.x < ns) {
    const int sl = threadIdx.x;
    const int p = S.par(sl);
    const bool local = p >= js0 && p < js1;
    sP[sl] = local ? p - js0 : -1;
    sZp[sl] = sA_;
    sH[sl] = (!local && p >= 0) ? sB_ : 0.0;
    sRho[sl] = (!local && p >= 0) ? p - ts0 : -1;
  }
  __syncthreads();
  for (int lv = lv0; lv < lv1; ++lv) {  // root level first
    const int la = S.lv(lv - lv0), lb = S.lv(lv - lv0 + 1);
    for (int j = la + threadIdx.x; j < lb; j += kPcThreads) {
      const int sl = j - js0;
      const int p = sP[sl];
      if (p >= 0) {
        sZp[sl] = sA[sl] + sB[sl] * sZp[p];
        sH[sl] = sB[sl] * sH[p];
        sRho[sl] = sRho[p];
      }
    }
    __syncthreads();
  }
}

// The u-independent part of one chain (lane state L, one pass): its cells' values and
// fluxes with zt = zb = 0.
// park: 2 CPL + 1 doubles per thread in LDS (kept there through the stores and the wait,
// not in registers: phase 2's registers are at the 128-VGPR budget of 1024 threads). Run by
// phase 1 (dir_up_v2) on its chain lane state: ch, L and vc = the cell inputs w_c
// (direct_cell_inputs), so the Thomas scans of M^{-1} b_q are not repeated.
template <int W, int CPL>
__device__ __forceinline__ void dir_sup_chain_core(const ChainLane<W, CPL>& ch,
                                                   const DirLane<W, CPL>& L, const double* vc,
                                                   double* park) {
  double zc[CPL], xq[CPL + 1];
  const double T = ch.T, iT = 1.0 / T;
  double a[CPL], bs[CPL], sa = 0.0, sb = 0.0;
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    a[t] = (T - ch.D[t]) * vc[t];
    bs[t] = ch.D[t] * vc[t];
    sa += a[t];
    sb += bs[t];
  }
  const double ia = seg_incl_scan<W>(sa), ibv = seg_incl_scan<W>(sb);
  const double Atot = seg_sum<W>(sa);
  double pa_ = ia - sa, pb_ = ibv - sb;
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    pa_ += a[t];
    const double suffix = Atot - pa_ + a[t];
    const double prefix = pb_;
    pb_ += bs[t];
    const double Dk = ch.D[t];
    zc[t] = ch.valid[t] ? (Dk * iT * suffix + (T - Dk) * iT * prefix) - ch.mo * vc[t] : 0.0;
  }
  direct_flux_cons<W, CPL>(ch, L.flip, L.bc, L.bq, L.bN, 0.0, 0.0, xq);
#pragma unroll
  for (int t = 0; t < CPL; ++t) park[t * kPcThreads + threadIdx.x] = zc[t];
#pragma unroll
  for (int t = 0; t <= CPL; ++t) park[(CPL + t) * kPcThreads + threadIdx.x] = xq[t];
}

// Wave 0's chains' u-independent part (sup_wslots: deferred from phase 1 into the wait; the
// cell inputs wait in the park's cell slots)
template <int W, int CPL>
__device__ __forceinline__ void dir_sup_core_wave0(const PcArgs& pa, const DirLane<W, CPL>& L,
                                                   bool active, double* park) {
  if (threadIdx.x >= 64) return;
  ChainLane<W, CPL> ch;
  dir_lane_chain<W, CPL>(pa, L, active, ch);
  double vc[CPL];
#pragma unroll
  for (int t = 0; t < CPL; ++t) vc[t] = park[t * kPcThreads + threadIdx.x];
  dir_sup_chain_core<W, CPL>(ch, L, vc, park);
}

// After the top values (sTop by top position): every slot's value (sZ over sZp), then the
// chains' values from their end values, the fused true residual of those final values, the
// chains' posts and the job's partial sums (rpart). park: dir_sup_chain_core's values on entry,
// the final ones on return (stored by dir_sup_store_x after the hand-off).
template <int W, int CPL>
__device__ __forceinline__ void dir_sup_finish(const PcArgs& pa, const DirStep& da, double* lds,
                                               const double* sTop, const JobStash& S,
                                               const DirLane<W, CPL>& L, double* sup,
                                               double* park, int job) {
  double* sZ = sup + 2 * kCapS;  // (over sZp)
  const double* sH = sZ + kCapS;
  const int* sRho = reinterpret_cast<const int*>(sH + kCapS);
  double* sQt = lds;
  double* sQb = sQt + kCapC;
  __shared__ double s_w[2 * (kPcThreads / 64)];
  const int ts0 = pa.top_ts0;
  const int js0 = S.js0, js1 = S.js1, ns = js1 - js0;
  const int c0 = S.c0, c1 = S.c1;
  const int seg = threadIdx.x / W, l = threadIdx.x & (W - 1);
  const bool active = c0 + seg < c1;
  if ((int)threadIdx.x < ns) {
    const int sl = threadIdx.x;
    const int rho = sRho[sl];
    const double z = rho >= 0 ? sZ[sl] + sH[sl] * sTop[rho] : sZ[sl];
    sZ[sl] = z;
    if (!NX_LEDGER(da, 4)) da.x[S.lam(sl)] = z;
  }
  __syncthreads();
  NX_DSTAMP(21);
  const int up = active ? S.cup(seg) : -1, lo = active ? S.clo(seg) : -1;
  const double zt = up < 0 ? 0.0 : (up >= js0 && up < js1) ? sZ[up - js0] : sTop[up - ts0];
  const double zb = lo < 0 ? 0.0 : (lo >= js0 && lo < js1) ? sZ[lo - js0] : sTop[lo - ts0];
  ChainLane<W, CPL> ch;
  dir_lane_chain<W, CPL>(pa, L, active, ch);
  double zc[CPL], xq[CPL + 1];
#pragma unroll
  for (int t = 0; t < CPL; ++t) zc[t] = park[t * kPcThreads + threadIdx.x];
#pragma unroll
  for (int t = 0; t <= CPL; ++t) xq[t] = park[(CPL + t) * kPcThreads + threadIdx.x];
  {
    const double T = ch.T, iT = 1.0 / T;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      const double Dk = ch.D[t];
      if (ch.valid[t]) zc[t] = zc[t] + (zt * (T - Dk) * iT + zb * Dk * iT);
    }
    const double sg = L.flip ? -1.0 : 1.0;
    const double dq0 = (sg * (zt - zb)) / T;
#pragma unroll
    for (int t = 0; t < CPL; ++t)
      if (ch.valid[t]) xq[t] = xq[t] + dq0;
    if (ch.has_last) xq[CPL] = xq[CPL] + dq0;
  }
  double rr = 0.0, bb = 0.0;
  direct_residual<W, CPL, false>(pa, ch, active, L.flip, L.bc, L.bq, L.bN, zc, xq, zt, zb, L.mo,
                                 rr, bb, sQt, sQb, seg);
#pragma unroll
  for (int t = 0; t < CPL; ++t) park[t * kPcThreads + threadIdx.x] = zc[t];
#pragma unroll
  for (int t = 0; t <= CPL; ++t) park[(CPL + t) * kPcThreads + threadIdx.x] = xq[t];
  const int post_t = active ? S.cpt(seg) : -1, post_b = active ? S.cpb(seg) : -1;
  if (active && l == 0 && post_t >= 0) st_wt(da.post + post_t, sQt[seg]);
  if (ch.has_last && post_b >= 0) st_wt(da.post + post_b, sQb[seg]);
  __syncthreads();
  NX_DSTAMP(22);
  // multiplier rows of the junctions whose chains are all in this job (b_lambda = 0)
  if ((int)threadIdx.x < ns && S.rloc(threadIdx.x)) {
    const int sl = threadIdx.x;
    const int pc = S.pchain(sl);
    double acc = pc >= 0 ? sQb[pc - c0] : 0.0;
    for (int i = S.dcoff(sl); i < S.dcoff(sl + 1); ++i) acc += sQt[S.sdc(i - S.dc0) - c0];
    const double rl = 0.0 - acc;
    rr += rl * rl;
  }
  rr = wave_sum(rr);
  bb = wave_sum(bb);
  if ((threadIdx.x & 63) == 0) {
    s_w[threadIdx.x >> 6] = rr;
    s_w[kPcThreads / 64 + (threadIdx.x >> 6)] = bb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tr = s_w[0], tb = s_w[kPcThreads / 64];
    for (int i = 1; i < kPcThreads / 64; ++i) {
      tr += s_w[i];
      tb += s_w[kPcThreads / 64 + i];
    }
    st_wt(pa.rpart + job, tr);
    st_wt(pa.rpart + pa.n_jobs + job, tb);
  }
}

// The chain lane's final values into x (after the phase-2 hand-off): cells, fluxes, q_N.
template <int W, int CPL>
__device__ __forceinline__ void dir_sup_store_x(const PcArgs& pa, const DirStep& da,
                                                const DirLane<W, CPL>& L, bool active,
                                                const double* park) {
  if (!active || NX_LEDGER(da, 4)) return;
  const double* zc = park + threadIdx.x;
  const double* xq = park + CPL * kPcThreads + threadIdx.x;
  const int N = pa.N;
  const int l = threadIdx.x & (W - 1);
  const int flip = L.flip;
  double* __restrict__ x = da.x + (int64_t)L.e * (2 * N + 1);
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    const int k = l * CPL + t;
    if (k >= N) continue;
    x[2 * (flip ? N - 1 - k : k) + 1] = zc[t * kPcThreads];
    x[2 * (flip ? N - k : k)] = xq[t * kPcThreads];
  }
  if (l == (N - 1) / CPL) x[flip ? 0 : 2 * N] = xq[CPL * kPcThreads];
}

// The assembly's stores of one workgroup: a share of job jb's multiplier rows (+-1 values,
// zero rhs: indices jb * kPcThreads + k, k < kPcThreads, then every nj * kPcThreads), then jb's
// chains [cs, ce) -- from the kept lanes (keep: this workgroup's own single pass, chain cs +
// group) or re-assembled from their records (chain cb + group - g0 per pass). Only the lane
// groups [g0, g1) store (the others -- whole waves -- stay free of outstanding stores, so their
// polls and loads are not queued behind them).
template <int W, int CPL, bool UNIT = false>
__device__ __forceinline__ void dir_stores_v2(const PcArgs& pa, const DirStep& da, int jb, bool lm,
                                              int cs, int ce, bool keep, DirLane<W, CPL>& L,
                                              int g0 = 0, int g1 = kPcThreads / W) {
  const int nj = pa.n_jobs;
  const int grp = (int)threadIdx.x / W;
  const bool mine = grp >= g0 && grp < g1;
  if (lm && mine) {
    const int64_t nlm = da.nnz_lm > da.B ? da.nnz_lm : da.B;
    const int nthr = (g1 - g0) * W;
    for (int k = (int)threadIdx.x - g0 * W; k < kPcThreads; k += nthr)
      for (int64_t i = (int64_t)jb * kPcThreads + k; i < nlm; i += (int64_t)nj * kPcThreads) {
        if (i < da.nnz_lm && !NX_LEDGER(da, 16)) da.val_lm[i] = da.lm_val[i];
        if (i < da.B && !NX_LEDGER(da, 16)) da.rhs_lm[i] = 0.0;
      }
  }
  if (keep) {
    if (mine) dir_chain_store<W, CPL, UNIT>(pa, da, cs + grp < ce, L);
    return;
  }
  const int per = g1 - g0;
  for (int cb = cs; cb < ce; cb += per) {
    const int c = cb + grp - g0;
    if (mine) {
      ChainRec r;
      chain_rec_load(da, c, c < ce, r);
      dir_chain_asm_rec<W, CPL>(pa, r, c < ce, L);
      dir_chain_store<W, CPL, UNIT>(pa, da, c < ce, L);
    }
  }
}

// k_dir_step's waiting workgroups leave the stores of their first kDirFreeWaves waves until
// after phase 2: those waves poll for the top values and load them without waiting for the
// drain of the others' stores. The top solver's assembly is stored by the first workgroups to
// arrive (helpers), one chain per wave on the other waves: kDirHelpChains chains each.
constexpr int kDirFreeWaves = 4;
constexpr int kDirHelpChains = kPcThreads / 64 - kDirFreeWaves;
// dynamic LDS of k_dir_step: at most this (the static __shared__ words -- flags, the partial
// sums of phase 2 and the publish -- take the rest of the CU's 160 KiB)
constexpr int kDirLdsMax = 160 * 1024 - 2048;

// The chain records of k_dir_step (crec / ci) from the edge arrays: run when the
// decomposition or the coefficients (R, f, boundary values) change, not per step.
__global__ __launch_bounds__(256) void k_chain_rec(const int* __restrict__ chain_edge,
                                                   const int* __restrict__ chain_flip, int64_t nc,
                                                   const double* __restrict__ edge_x,
                                                   const double* __restrict__ edge_R,
                                                   const double* __restrict__ edge_f, double f,
                                                   const double* __restrict__ edge_bc,
                                                   const int* __restrict__ edge_lm,
                                                   const int* __restrict__ edge_seg,
                                                   double* __restrict__ crec, int* __restrict__ ci) {
  const int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (c >= nc) return;
  const int e = chain_edge[c];
  double* r = crec + 10 * c;
  for (int i = 0; i < 6; ++i) r[i] = edge_x[6 * (int64_t)e + i];
  r[6] = edge_R[e];
  r[7] = edge_f ? edge_f[e] : f;
  r[8] = edge_bc[2 * (int64_t)e];
  r[9] = edge_bc[2 * (int64_t)e + 1];
  ci[4 * c] = e;
  ci[4 * c + 1] = (chain_flip[c] & 1) | ((edge_lm[2 * (int64_t)e] >= 0 ? 1 : 0) << 1);
  ci[4 * c + 2] = edge_seg[e];
  ci[4 * c + 3] = edge_seg[e + 1] - edge_seg[e];
}

// ---- the device-side exchange between ranks (k_dir_xr / k_dir_xg) ---------------------
__device__ __forceinline__ void st_sys(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double ld_sys(const double* p) {
  return __builtin_bit_cast(
      double, __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<double*>(p)),
                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}

// rank q's abort word in this rank's mailbox: (reasons << 32) | the tag of the launch that
// gave up; 0 while q never gave up
__device__ __forceinline__ unsigned long long xr_abort_of(const DirStep& da, int q) {
  return __hip_atomic_load(reinterpret_cast<unsigned long long*>(da.xself.fl + 2 * da.xP) + q,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One lane of a rank that gives up an exchange step: the reasons for the host (sync[5]) and
// (reasons, this launch's tag) in its abort word in every other rank's mailbox, so their
// exchanges waiting on it fail at once instead of waiting out their bound, and their hosts
// know how far it got (xr_host_finish).
__device__ __forceinline__ void xr_give_up(const DirStep& da, unsigned why) {
  __hip_atomic_fetch_or(da.sync + 5, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long w = ((unsigned long long)why << 32) | da.xtag;
  for (int q = 0; q < da.xP; ++q)
    if (q != da.xrank)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(da.xpeers[q].fl + 2 * da.xP) + da.xrank,
                         w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Exchange round `which` (0: coarse partials, 1: residual partials) of one workgroup: this
// rank's n doubles (src, LDS) and its launch tag (the slot's last double) into its slot of
// every rank's mailbox, then -- after every storing wave's vmcnt(0) and a barrier -- its
// flag at every rank (tagged with the launch); then this rank's P flags polled (bounded,
// and failing at once on a raised abort word) and the P slots summed in rank order (the
// same additions as k_group_sum: every rank gets the same bits) into dst (LDS), each slot's
// tag checked beside the sums. False: a rank's flag never came, another rank gave up, or a
// slot held another launch's data; this rank's abort is then raised everywhere.
//
// Ordering (the advisor's r04 finding): the slots and the flag are system-scope atomic
// stores (write-through to the coherence point) and vmcnt(0) retires the slots' stores
// before any flag store issues -- what a system-scope release does for atomic data (its
// L2 write-back covers plain stores only, and there are none here). The reader's slot loads
// are system-scope atomic loads (they bypass the non-coherent caches), issued after the
// flag load returned (a barrier orders the polling lanes before every loading lane) -- the
// acquire's ordering for atomic loads (its cache invalidation covers plain loads only). The
// slot tags check it: a reordered slot cannot carry this launch's tag.
__device__ __forceinline__ bool xr_allsum(const DirStep& da, int which, const double* src, int n,
                                          double* dst) {
  __shared__ unsigned sWhy;
  const int P = da.xP, r = da.xrank, ld = which ? da.xld2 : da.xld1;
  const double tagd = __builtin_bit_cast(double, (unsigned long long)da.xtag);
  for (int q = 0; q < P; ++q) {
    double* mb = (which ? da.xpeers[q].mb2 : da.xpeers[q].mb1) + (int64_t)r * ld;
    for (int i = threadIdx.x; i < n; i += kPcThreads) st_sys(mb + i, src[i]);
    if (threadIdx.x == kPcThreads - 1) st_sys(mb + ld - 1, tagd);
  }
  vm_drain();
  if (threadIdx.x == 0) sWhy = 0u;
  __syncthreads();
  if ((int)threadIdx.x < P)
    __hip_atomic_store(da.xpeers[threadIdx.x].fl + which * P + r, da.xtag, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  if ((int)threadIdx.x < P) {
    unsigned why = which ? kXrFail2 : kXrFail1;
    const unsigned polls = da.xpoll[which];
    for (unsigned k = 0; k < polls; ++k) {
      if (__hip_atomic_load(da.xself.fl + which * P + threadIdx.x, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_SYSTEM) == da.xtag) {
        why = 0u;
        break;
      }
      if ((unsigned)xr_abort_of(da, threadIdx.x) == da.xtag) {  // rank q gave up this launch
        why |= kXrFailAbort;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (why) atomicOr(&sWhy, why);
  }
  __syncthreads();
  if (sWhy == 0u) {
    const double* mine = which ? da.xself.mb2 : da.xself.mb1;
    for (int i = threadIdx.x; i < n; i += kPcThreads) {
      double v = 0.0;
      for (int q = 0; q < P; ++q) v += ld_sys(mine + (int64_t)q * ld + i);
      dst[i] = v;
    }
    if ((int)threadIdx.x < P &&
        __builtin_bit_cast(unsigned long long, ld_sys(mine + (int64_t)threadIdx.x * ld + ld - 1)) !=
            (unsigned long long)da.xtag)
      atomicOr(&sWhy, (which ? kXrFail2 : kXrFail1) | kXrFailTag);
    __syncthreads();
  }
  const unsigned why = sWhy;
  if (why != 0u && threadIdx.x == 0) xr_give_up(da, why);
  return why == 0u;
}

// The coarse step's static set-up of this thread's top slot (coarse_top_pre's indices),
// loaded with the top part's own indices, and its parent chain's T with the top part's
// inputs (posted by phase 1): nothing of the coarse step waits for a load after the exchange.
struct CoarseIdx {
  int k, par, pch, lvo, cw0, cw1;
  double T;
};
__device__ __forceinline__ void coarse_idx_load(const PcArgs& pa, CoarseIdx& c) {
  const int sl = threadIdx.x, ts0 = pa.top_ts0, nt = pa.top_nt;
  c.lvo = sl <= pa.n_top_lvl ? pa.top_lvl_off[sl] : 0;
  const bool cw = pa.c_wave && sl < pa.n_coarse;
  c.cw0 = cw ? pa.c_wave[2 * sl] : 0;
  c.cw1 = cw ? pa.c_wave[2 * sl + 1] : 0;
  c.k = sl < nt ? pa.slot_cidx[ts0 + sl] : -1;
  c.par = sl < nt ? pa.slot_parent[ts0 + sl] : -1;
  c.pch = sl < nt ? pa.slot_pchain[ts0 + sl] : -1;
  c.T = 1.0;
}
__device__ __forceinline__ void coarse_idx_val(const PcArgs& pa, CoarseIdx& c) {
  if (c.k < 0 && c.par >= 0 && c.pch >= 0) c.T = ld_wt(pa.chain_T + c.pch);
}

// The top part's solver after top_body<MULTI>: exchange 1 of the coarse partials (cbuf),
// the sums back into cbuf, the coarse forest and the top part's back-substitution
// (coarse_top_block, k_pc_coarse's arithmetic: coarse_top_pre's values, from LDS and the
// prefetched ci) into LDS, then the top values to slot_z (write-through: the rank's other
// workgroups read them) and to x.
// The top part's back-substitution from the coarse values (coarse_top_block's arithmetic
// and order per slot: the same bits) on the wave subtrees of pa.top_sub: the upper slots
// level by level (barriers), then every subtree by its wave, root first, the parent's value
// by shuffle. Per slot (LDS): D / J (top_body's sD / sJ), its parent (sPar), its parent
// chain's T and coarse index (ext, kk).
__device__ __forceinline__ void xr_top_back(const PcArgs& pa, const CoarsePre& cp, const TopLds& T,
                                            const TopPre& pre, const double* cZ, double* tZ,
                                            double* ext, int* kk) {
  const int nt = pa.top_nt, sl = threadIdx.x;
  if (sl < nt) {
    ext[sl] = cp.T;
    kk[sl] = cp.k;
  }
  __syncthreads();
  const bool upper = sl < nt && pre.w[0] < 0;
  const int ulv = upper ? (pre.w[0] & 0xff) : -1;
  const int par = sl < nt ? T.sPar[sl] : -1;
  for (int lv = 0; lv < pa.top_sub_nup; ++lv) {
    if (ulv == lv) {
      double zj;
      if (cp.k >= 0) {
        zj = cZ[cp.k];
      } else {
        double num = cp.J;
        if (par >= 0) num += tZ[par] / cp.T;
        zj = num / cp.D;
      }
      tZ[sl] = zj;
    }
    __syncthreads();
  }
  if (pre.ldep > 0) {
    const int lsl = pre.ls;
    const int lvl = (pre.lw[0] >> 6) & 0xff, plane = (pre.lw[0] >> 18) & 63;
    const int k = lsl >= 0 ? kk[lsl] : -1, pq = lsl >= 0 ? T.sPar[lsl] : -1;
    const double J = lsl >= 0 ? T.sJ[lsl] : 0.0, D = lsl >= 0 ? T.sD[lsl] : 1.0;
    const double Tq = lsl >= 0 ? ext[lsl] : 1.0;
    double zq = 0.0;
    for (int q = 0; q < pre.ldep; ++q) {
      const double zp = __shfl(zq, plane);
      if (lvl == q && lsl >= 0) {
        if (k >= 0) {
          zq = cZ[k];
        } else {
          const double zpar = q == 0 ? (pq >= 0 ? tZ[pq] : 0.0) : zp;
          double num = J;
          if (pq >= 0) num += zpar / Tq;
          zq = num / D;
        }
      }
    }
    if (lsl >= 0) tZ[lsl] = zq;
  }
  __syncthreads();
}

__device__ __forceinline__ bool xr_coarse(const PcArgs& pa, const DirStep& da, const TopLds& T,
                                          const CoarseIdx& ci, const TopPre& pre, double* ext) {
  __shared__ double xb[2 * 3 * kCapCoarseLds];
  const int nC = pa.n_coarse, n1 = 3 * nC;
  for (int i = threadIdx.x; i < n1; i += kPcThreads) xb[i] = ld_wt(pa.cbuf + i);
  __syncthreads();
  NX_DSTAMP(42);
  if (!xr_allsum(da, 0, xb, n1, xb + n1)) return false;
  NX_DSTAMP(43);
  if (!pa.c_wave) {  // (pc_coarse_lds reads the sums from cbuf)
    for (int i = threadIdx.x; i < n1; i += kPcThreads) pa.cbuf[i] = xb[n1 + i];
    vm_drain();
    __syncthreads();
  }
  const int ts0 = pa.top_ts0, nt = pa.top_nt, sl = threadIdx.x;
  CoarsePre cp;  // (coarse_top_pre's values: the top slots' D / J from top_body's LDS)
  cp.k = ci.k;
  cp.par = ci.k < 0 ? ci.par : -1;
  cp.J = ci.k < 0 && sl < nt ? T.sJ[sl] : 0.0;
  cp.D = ci.k < 0 && sl < nt ? T.sD[sl] : 1.0;
  cp.T = ci.k < 0 && ci.par >= 0 ? ci.T : 1.0;
  cp.lvo = ci.lvo;
  cp.cw0 = ci.cw0;
  cp.cw1 = ci.cw1;
  const bool cm = pa.c_wave && sl < nC;
  cp.cD = cm ? xb[n1 + sl] : 1.0;
  cp.cJ = cm ? xb[n1 + nC + sl] : 0.0;
  cp.cG = cm ? xb[n1 + 2 * nC + sl] : 0.0;
  __syncthreads();  // (coarse_top_block overwrites T.sD0 / sJ0 / sGp / sY)
  if (pa.top_sub) {  // the coarse forest, then the top part by its wave subtrees
    if (pa.c_wave) {
      coarse_wave_solve_rcp(pa, cp.cw0, cp.cw1, cp.cD, cp.cJ, cp.cG, T.sGp);
      __syncthreads();
    } else {
      pc_coarse_lds(pa, T.sD0, T.sJ0, T.sGp);
    }
    NX_DSTAMP(46);
    xr_top_back(pa, cp, T, pre, T.sGp, T.sY, ext, reinterpret_cast<int*>(ext + nt + 1));
    NX_DSTAMP(47);
  } else {
    coarse_top_block(pa, cp, T.sD0, T.sJ0, T.sGp, T.sY, T.sOff);
  }
  for (int i = threadIdx.x; i < nt; i += kPcThreads) {
    const double zj = T.sY[i];
    st_wt(pa.slot_z + ts0 + i, zj);
    if (!NX_LEDGER(da, 4)) da.x[T.sLam[i]] = zj;
  }
  return true;
}

// The publisher of a rank of several (k_dir_xr / k_dir_xg): dir_publish_fused's sums of the
// rank's own rows, the cut rows' shares of this rank (the last xK post ranges), exchange 2,
// then every rank the same relres: the rows' ||r||^2 summed in rank order plus the cut
// rows' r^2 in index order (r = 0 - the ranks' shares: b = 0 on the multiplier rows).
__device__ __forceinline__ bool dir_publish_xr(const PcArgs& pa, const DirStep& da, int lo0, int lo1) {
#pragma clang fp contract(off)
  __shared__ double s_r[kPcThreads / 64], s_b[kPcThreads / 64];
  __shared__ double xs[2 * (2 + kCapCoarseLds)];
  const int nj = pa.n_jobs, K = da.xK, nl = da.n_left;
  double rr = 0.0, bb = 0.0;
  for (int i = threadIdx.x; i < nj; i += kPcThreads) {
    rr += ld_wt(pa.rpart + i);
    bb += ld_wt(pa.rpart + nj + i);
  }
  for (int i = threadIdx.x; i < nl; i += kPcThreads) {
    const bool pre = i == (int)threadIdx.x;
    const int k0 = pre ? lo0 : da.left_off[i], k1 = pre ? lo1 : da.left_off[i + 1];
    const double rv = 0.0 - post_sum(da.post, k0, k1);  // b = 0 on the multiplier rows
    rr += rv * rv;
  }
  for (int k = threadIdx.x; k < K; k += kPcThreads)  // this rank's shares of the cut rows
    xs[2 + k] = post_sum(da.post, da.left_off[nl + k], da.left_off[nl + k + 1]);
  rr = wave_sum(rr);
  bb = wave_sum(bb);
  if ((threadIdx.x & 63) == 0) {
    s_r[threadIdx.x >> 6] = rr;
    s_b[threadIdx.x >> 6] = bb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    rr = 0.0;
    bb = 0.0;
    for (int w = 0; w < kPcThreads / 64; ++w) {
      rr += s_r[w];
      bb += s_b[w];
    }
    xs[0] = rr;
    xs[1] = bb;
  }
  __syncthreads();
  double* ys = xs + 2 + K;
  NX_DSTAMP(44);
  if (!xr_allsum(da, 1, xs, 2 + K, ys)) return false;
  NX_DSTAMP(45);
  {  // a rank that gave up this launch after its flag reached this one: publishing nothing
     // keeps the ranks together (x is final; the host finishes exchange 2, xr_host_finish)
    __shared__ int sAb;
    if (threadIdx.x == 0) sAb = 0;
    __syncthreads();
    if ((int)threadIdx.x < da.xP && (unsigned)xr_abort_of(da, threadIdx.x) == da.xtag) sAb = 1;
    __syncthreads();
    if (sAb) {
      if (threadIdx.x == 0) xr_give_up(da, kXrFail2 | kXrFailAbort);
      return false;
    }
  }
  if (threadIdx.x == 0) {
    rr = ys[0];
    for (int k = 0; k < K; ++k) {
      const double rk = 0.0 - ys[2 + k];
      rr += rk * rk;
    }
    bb = ys[1];
    da.bbst[0] = bb;
    MrState st{};
    st.beta1 = sqrt(bb);
    st.relres = bb > 0.0 ? sqrt(rr / bb) : sqrt(rr);
    st.rtol = da.rtol;
    st.it = 1;
    st.done = 1;
    st.converged = st.relres <= da.rtol ? 1 : 0;
    publish_wt(st, da.seq_next, da.seq, da.mirror);
  }
  return true;
}

// The fused direct step of one rank (k_dir_step) or, XR, of one rank of several (k_dir_xr:
// one launch per GPU; k_dir_xg: every rank of an in-process group in one launch): the top
// part then ends with this rank's coarse partials, the ranks exchange and sum them
// (xr_allsum), the top part's solver finishes the coarse forest and the top values, and
// the publisher exchanges the residual's partials and the cut rows' shares the same way.
template <int W, int CPL, bool XR, bool SUP>
__device__ __forceinline__ void dir_step_body(const PcArgs& pa, const DirStep& da, int job) {
  extern __shared__ double dsm[];
  __shared__ int sFlag, sTopJob, sIdx;
  int* stash = reinterpret_cast<int*>(dsm);  // the job's statics (fixed offsets)
  double* smem = dsm + kStashDbl;            // phase 1 / the top part / phase 2
  double* sTop = smem + da.lds_main;         // the top part's values (phase 2 reads them)
  const int nj = pa.n_jobs;
  const unsigned last = da.epoch * (unsigned)nj + (unsigned)(nj - 1);
  const unsigned tag = (da.epoch + 1u) << 10;  // the top solver's announcement (job < 1024)
  constexpr int G = kPcThreads / W;
  NX_DSTAMP(0);
  JobStash S;
  ChainRec rec;
  {
    StashRegs R;
    job_stash_load<W>(pa, da, job, stash, S, R);
    chain_rec_load(da, S.c0 + (int)threadIdx.x / W, S.c0 + (int)threadIdx.x / W < S.c1, rec);
    job_stash_store(S, R, min(S.c1 - S.c0, G));
  }
  __syncthreads();
  const int c0 = S.c0, c1 = S.c1;
  // the job's chains in one pass: the assembly's stores wait until this workgroup has handed
  // over its top inputs (they fill the wait for the top values instead of delaying it), and
  // phase 2 runs on phase 1's registers
  // (SUP: launched only when every job fits one pass, dstep_multi false -- its instantiation
  // carries no several-pass code)
  const bool keep = SUP || c1 - c0 <= G;
  // phase 2 by superposition (dir_sup_*: one chain pass; the top solver then stores its own
  // assembly after its phase 2, no helpers)
  // (compiled in only where it is launched, CPL <= 2: its code kept beside the plain phase 2
  // costs the other instantiations registers they do not have)
  const bool sup = SUP;
  bool sup_s = false;  // this workgroup formed its slots' z_p / H (dir_sup_slots)

  // the slots' back-substitution coefficients (phase 1's sA_ / sB_, thread = slot) wait in LDS
  // (sup: the slots' region, kDirLdsSupSlots), not in registers (the top solver's would stay
  // live through the top part); the chains' u-independent values in the park after it
  double* sup_lds = sTop + da.lds_top;
  double* park = sup_lds + kDirLdsSupSlots;
  // sup & 4: the chain records and every lane's cell masses and cell rhs in LDS too (the top
  // solver rebuilds its lanes from them after the top part -- no loads under the store
  // stream, no second assembly -- and so do the stores left for the kernel's tail)
  double* rec_lds = sup && (da.sup & 4) ? park + (2 * CPL + 1) * kPcThreads : nullptr;
  double* lpark = rec_lds ? rec_lds + kRecLds * G : nullptr;
  // (keep) helpers store the top solver's assembly; the free waves' lane groups [0, gF).
  // Superposition: only wave 0 (the poll) stays free of stores -- the waiting workgroups'
  // values come after their stores have long drained, so waves 1-3 store in the wait too
  // Superposition also spreads the top solver's chains thinner: one chain per helper, stored
  // by the helper's wave 0 in the kernel's tail (after x: its stores would hold up the poll
  // for the top values and their loads behind them; no barrier either)
  const int fw = sup ? 1 : kDirFreeWaves, hc = sup ? 1 : kPcThreads / 64 - fw;
  const int nh = min(nj - 1, (G + hc - 1) / hc);
  const int gF = fw * 64 / W;
  DirLane<W, CPL> L;
  double sA_ = 0.0, sB_ = 0.0;
  const int nt = pa.top_nt, ts0 = pa.top_ts0;
  if (rec_lds) rec_to_lds<W>(rec_lds, c0 + (int)threadIdx.x / W < c1, rec);
  dir_up_v2<W, CPL>(pa, da, smem, S, rec, L, sA_, sB_, sup ? park : nullptr);
  if (lpark) {
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      lpark[t * kPcThreads + threadIdx.x] = L.mo[t];
      lpark[(CPL + t) * kPcThreads + threadIdx.x] = L.bc[t];
    }
  }
  if ((int)threadIdx.x < kCapS) {
    sup_lds[threadIdx.x] = sA_;
    sup_lds[kCapS + threadIdx.x] = sB_;
  }
  NX_DSTAMP(35);
  bool late_store = false;  // the top solver stores its own assembly after phase 2 (no helpers)
  bool helper = false;      // (superposition) a helper storing its top solver chain in the tail
  bool defer_free = false;  // a waiting workgroup's free waves store theirs after phase 2
  const bool lane_on = c0 + (int)threadIdx.x / W < c1;
  if (nt > 0) {  // hand-off 1: the top part's inputs -> the last workgroup -> its values
    vm_drain();
    __syncthreads();
    NX_DSTAMP(1);
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(da.sync, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      sFlag = old == last ? 1 : 0;
      sIdx = (int)(old - da.epoch * (unsigned)nj);  // this workgroup's arrival order
      if (sFlag && keep && nh > 0)  // tell the helpers whose assembly to store
        __hip_atomic_store(da.sync + 4, tag | (unsigned)job, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (sFlag) {
      // this workgroup re-assembles its lanes after the top part (kept registers would stay
      // live through the solve, past the register budget); its assembly is stored by the
      // helpers (keep) or after its phase 2 (one job) or, with several chain passes (its phase
      // 2 reloads b and dq), right after the top part
      late_store = keep && nh == 0;
      const int ct = nt + 1, cdc = pa.top_ndc > 0 ? pa.top_ndc : 1;  // this top part's sizes
      double* t = smem;
      TopLds T;
      T.sD0 = t; t += ct;
      T.sJ0 = t; t += ct;
      T.sD = t; t += ct;
      T.sJ = t; t += ct;
      T.sGp = t; t += ct;
      T.sY = t; t += ct;
      T.sG = t; t += cdc;
      T.sDD = t; t += cdc;
      T.sDJ = t; t += cdc;
      int* u = reinterpret_cast<int*>(t);
      T.sPar = u; u += ct;
      T.sLam = u; u += ct;
      T.sOff = u; u += ct + 1;
      T.sChild = u; u += cdc;
      T.sLv = u;
      TopPre pre;
      top_pre_idx(pa, pre);
      CoarseIdx ci;
      if constexpr (XR) coarse_idx_load(pa, ci);
      top_pre_val<true>(pa, nullptr, pre);
      if constexpr (XR) coarse_idx_val(pa, ci);
      NX_DSTAMP(6);
      if constexpr (XR) {
        // the rank's top part up to its coarse partials [D | J | G] (pc_coarse_partials: in
        // cbuf; the top slots' D / J in slot_D / slot_J), then the exchange, then the coarse
        // forest and the top part's back-substitution (k_pc_coarse's arithmetic: the same
        // bits as the separate launches) from the sums
        top_body<true, true>(pa, nullptr, nullptr, da.x, nullptr, nullptr, 0, nullptr, nullptr,
                             kModeDirect, T, false, pre);
        vm_drain();
        __syncthreads();
        NX_DSTAMP(41);
        // (xr_top_back's per-slot scratch after the top part's arrays; sLv is the last)
        double* ext = reinterpret_cast<double*>(T.sLv + ((pa.n_top_lvl + 2) & ~1));
        if (!xr_coarse(pa, da, T, ci, pre, ext)) {
          if (threadIdx.x == 0) {  // the waiters leave at once (no top values will come)
            __hip_atomic_fetch_add(da.sync + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(da.sync + 2, kXrTopFailed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          return;
        }
      } else {
        top_body<false, true>(pa, nullptr, nullptr, da.x, nullptr, nullptr, 0, nullptr, nullptr,
                              kModeDirect, T, false, pre);
      }
      NX_DSTAMP(7);
      vm_drain();
      __syncthreads();
      NX_DSTAMP(5);
      if (threadIdx.x == 0)
        __hip_atomic_store(da.sync + 2, da.epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!keep) {
        dir_stores_v2<W, CPL>(pa, da, job, true, c0, c1, false, L);
        vm_drain();  // (its phase 2 reads them back)
      } else {  // its lanes again: not kept through the solve
        if (lpark) {
          lane_from_lds<W, CPL>(pa, rec_lds, lpark, lane_on, L);
        } else {
          chain_rec_load(da, fresh_chain<W>(c0), lane_on, rec);
          dir_chain_asm_rec<W, CPL>(pa, rec, lane_on, L);
        }
        if (sup) {  // its slots' z_p / H and wave 0's chains' part now (not before the top
                    // part: on its own path either way, and there it delayed the top values)
          dir_sup_slots<W, CPL>(pa, sup_lds, S);
          if (sup_wslots(S)) dir_sup_core_wave0<W, CPL>(pa, L, lane_on, park);
          sup_s = true;
        }
      }
    } else {
      // the first nh workgroups to arrive store the top solver's assembly first (they have
      // the most slack; their polls come before any store of theirs, so they see the
      // announcement at once), then their own
      if (!sup && keep && nh > 0 && sIdx < nh) {
        if (threadIdx.x == 0) {
          int who = -1;
          for (unsigned k = 0; k < da.polls; ++k) {
            const unsigned v = __hip_atomic_load(da.sync + 4, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            if ((v >> 10) == (tag >> 10)) {
              who = (int)(v & 1023u);
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          sTopJob = who;
        }
        __syncthreads();
        const int tj = sTopJob, hh = sIdx;
        if (tj >= 0) {  // helper hh: its share of the top solver's chains (+ helper 0 its rows)
          // one chain per wave (64 lanes: a chain's segment in a few whole-line store rounds)
          constexpr int CH = (W * CPL + 63) / 64;
          const int4 th = *reinterpret_cast<const int4*>(da.job_hdr + kJobHdr * (int64_t)tj);
          DirLane<64, CH> Lh;
          for (int cs = th.x + hh * hc; cs < th.y; cs += nh * hc)
            dir_stores_v2<64, CH, true>(pa, da, tj, hh == 0 && cs < th.x + hc, cs,
                                        min(th.y, cs + hc), false, Lh, fw, kPcThreads / 64);
        }
      }
      // superposition: the slots' z_p / H and wave 0's chains' part (one wave, the free one,
      // when they fit) in the wait
      if (sup) {
        dir_sup_slots<W, CPL>(pa, sup_lds, S);
        if (sup_wslots(S)) dir_sup_core_wave0<W, CPL>(pa, L, lane_on, park);
        sup_s = true;
        NX_DSTAMP(20);
      }
      helper = sup && nh > 0 && sIdx < nh;
      // own stores (unit stride: hidden in the wait), but not the free waves' (keep)
      dir_stores_v2<W, CPL, true>(pa, da, job, true, c0, c1, keep, L, keep ? gF : 0);
      defer_free = keep;
      if (!keep) vm_drain();  // (several passes: its phase 2 reads them back)
      NX_DSTAMP(8);
      if (threadIdx.x == 0) {
        int ok = 0;
        for (unsigned k = 0; k < da.polls; ++k) {
          const unsigned v = __hip_atomic_load(da.sync + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (v == da.epoch + 1u) {
            ok = 1;
            break;
          }
          if (XR && v == kXrTopFailed) {  // the solver gave up its exchange
            ok = -1;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        if (ok == 0) {
          __hip_atomic_fetch_add(da.sync + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if constexpr (XR) xr_give_up(da, kXrFail1 | kXrFailLocal);
        }
        sFlag = ok > 0 ? 1 : -1;
      }
    }
    __syncthreads();
    if (sFlag < 0) return;  // the top values never came (the host sees no published state)
    NX_DSTAMP(2);
    for (int i = threadIdx.x; i < nt; i += kPcThreads) sTop[i] = ld_wt(pa.slot_z + ts0 + i);
    __syncthreads();
  } else {
    dir_stores_v2<W, CPL>(pa, da, job, true, c0, c1, keep, L);
    vm_drain();
    __syncthreads();  // (several passes: phase 2 reads the stored b and dq back)
  }
  int lo0 = 0, lo1 = 0;  // this thread's left row's post range (dir_publish_fused)
  if ((int)threadIdx.x < da.n_left) {
    lo0 = da.left_off[threadIdx.x];
    lo1 = da.left_off[threadIdx.x + 1];
  }
  if (sup) {
    if (!sup_s) {  // no top part: the slots now
      dir_sup_slots<W, CPL>(pa, sup_lds, S);
      if (sup_wslots(S)) dir_sup_core_wave0<W, CPL>(pa, L, lane_on, park);
      __syncthreads();
    }
    dir_sup_finish<W, CPL>(pa, da, smem, sTop, S, L, sup_lds, park, job);
  } else {
    const bool sl = (int)threadIdx.x < kCapS;
    dir_down_v2<W, CPL>(pa, da, smem, sTop, S, L, keep, sl ? sup_lds[threadIdx.x] : 0.0,
                        sl ? sup_lds[kCapS + threadIdx.x] : 0.0, job);
  }
  // hand-off 2: the residual partials and shares -> the last workgroup publishes
  NX_DSTAMP(25);
  vm_drain();
  __syncthreads();
  NX_DSTAMP(3);
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(da.sync + 1, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    sFlag = old == last ? 1 : 0;
  }
  __syncthreads();
  if (sFlag) {
    if constexpr (XR) {
      if (!dir_publish_xr(pa, da, lo0, lo1) && threadIdx.x == 0)
        __hip_atomic_fetch_add(da.sync + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      dir_publish_fused(pa, da, lo0, lo1);
    }
    NX_DSTAMP(4);
  }
  if (sup) dir_sup_store_x<W, CPL>(pa, da, L, lane_on, park);
  if (helper && threadIdx.x < 64) {  // helper: wave 0, one chain
    int who = -1;
    if ((threadIdx.x & 63) == 0)
      for (unsigned k = 0; k < da.polls; ++k) {
        const unsigned v = __hip_atomic_load(da.sync + 4, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        if ((v >> 10) == (tag >> 10)) {
          who = (int)(v & 1023u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    const int tj = __shfl(who, 0);
    if (tj >= 0) {
      constexpr int CH = (W * CPL + 63) / 64;
      const int4 th = *reinterpret_cast<const int4*>(da.job_hdr + kJobHdr * (int64_t)tj);
      DirLane<64, CH> Lh;
      for (int cs = th.x + sIdx; cs < th.y; cs += nh)
        dir_stores_v2<64, CH, true>(pa, da, tj, cs == th.x, cs, cs + 1, false, Lh, 0, 1);
    }
  }
  // (the kernel's end, not the published state, waits for these; re-assembled: L kept
  // through phase 2 would overflow the register budget there)
  // (lpark: from the LDS copies)
  if (late_store || (defer_free && (int)threadIdx.x / W < gF)) {
    if (lpark) {
      lane_from_lds<W, CPL>(pa, rec_lds, lpark, lane_on, L);
    } else {
      chain_rec_load(da, fresh_chain<W>(c0), lane_on, rec);
      dir_chain_asm_rec<W, CPL>(pa, rec, lane_on, L);
    }
    if (late_store) {  // one job: the top solver's own
      dir_stores_v2<W, CPL>(pa, da, job, true, c0, c1, true, L);
    } else {  // the free waves' chains
      dir_chain_store<W, CPL>(pa, da, lane_on, L);
    }
  }
  vm_drain();
  NX_DSTAMP(40);
}

// SUP: phase 2 by superposition (DirStep::sup; instantiated for CPL <= 2, sup_launch)
template <int W, int CPL, bool SUP = false>
__global__ __launch_bounds__(kPcThreads) void k_dir_step(PcArgs pa, DirStep da) {
  dir_step_body<W, CPL, false, SUP>(pa, da, blockIdx.x);
}

// one rank of several, one GPU each (RCCL ranks; the exchange over IPC-mapped peer memory)
template <int W, int CPL, bool SUP = false>
__global__ __launch_bounds__(kPcThreads) void k_dir_xr(PcArgs pa, DirStep da) {
  dir_step_body<W, CPL, true, SUP>(pa, da, blockIdx.x);
}

// every rank of an in-process group in ONE launch (all their workgroups co-resident, so
// the ranks' exchanges can wait for each other): workgroup -> (rank, job) by goff
template <int W, int CPL, bool SUP = false>
__global__ __launch_bounds__(kPcThreads) void k_dir_xg(const PcArgs* __restrict__ pas,
                                                       const DirStep* __restrict__ das,
                                                       const int* __restrict__ goff, int P) {
  int r = 0;
  while (r + 1 < P && (int)blockIdx.x >= goff[r + 1]) ++r;
  dir_step_body<W, CPL, true, SUP>(pas[r], das[r], (int)blockIdx.x - goff[r]);
}

// k_dir_team_up: the first half of the several-rank direct step (one rank's share, before
// the coarse all-reduce) in ONE launch: every workgroup assembles its chains' edges in
// registers and runs the up sweep (dir_up_fused<MULTI>: phase 1 of k_dir_step, with the
// slots' and chains' data stored for the down sweep), hands the top part's inputs over
// write-through and leaves after its assembly stores; the workgroup arriving last solves the
// rank's top part and builds its coarse partials [D | J | G] (top_body<MULTI, WT>: what
// k_pc_top_lds does), then re-assembles its own lanes and stores them. It replaces
// k_assemble_seg -> k_pc_up_lds (mode 3) -> k_pc_top_lds. No workgroup waits for another
// (the last arrival does the work), so any number of jobs may run; the arrival counter is
// reset by the last workgroup (graph replays launch it with the same arguments).
template <int W, int CPL>
__global__ __launch_bounds__(kPcThreads) void k_dir_team_up(PcArgs pa, DirStep da) {
  __shared__ double smem[kDirLds];
  __shared__ int sFlag;
  const int job = blockIdx.x;
  const int nj = pa.n_jobs;
  NX_DSTAMP(0);
  const int c0 = pa.job_chain_off[job], c1 = pa.job_chain_off[job + 1];
  const bool keep = c1 - c0 <= kPcThreads / W;
  DirLane<W, CPL> L;
  double sA_ = 0.0, sB_ = 0.0;
  // (the assembly's stores after the hand-off, re-assembled pass by pass with several
  // passes: the last arrival -- the top part's start -- comes sooner)
  dir_up_fused<W, CPL, true>(pa, da, smem, L, false, sA_, sB_);
  auto stores = [&]() { dir_stores_all<W, CPL>(pa, da, job, keep, L); };
  vm_drain();
  __syncthreads();
  NX_DSTAMP(1);
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(da.sync, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    sFlag = old == (unsigned)(nj - 1) ? 1 : 0;
  }
  __syncthreads();
  if (!sFlag) {
    dir_stores_all<W, CPL, true>(pa, da, job, keep, L);  // (unit stride: see dir_chain_store)
    NX_DSTAMP(8);
    return;
  }
  if (pa.top_nt > 0) {
    double* t = smem;
    TopLds T;
    T.sD0 = t; t += kCapT;
    T.sJ0 = t; t += kCapT;
    T.sD = t; t += kCapT;
    T.sJ = t; t += kCapT;
    T.sGp = t; t += kCapT;
    T.sY = t; t += kCapT;
    T.sG = t; t += kCapTDC;
    T.sDD = t; t += kCapTDC;
    T.sDJ = t; t += kCapTDC;
    int* u = reinterpret_cast<int*>(t);
    T.sPar = u; u += kCapT;
    T.sLam = u; u += kCapT;
    T.sOff = u; u += kCapT + 1;
    T.sChild = u; u += kCapTDC;
    T.sLv = u;
    TopPre pre;
    top_pre_idx(pa, pre);
    top_pre_val<true>(pa, nullptr, pre);
    NX_DSTAMP(6);
    top_body<true, true>(pa, nullptr, nullptr, da.x, nullptr, nullptr, 0, nullptr, nullptr,
                         kModeDirect, T, false, pre);
  }
  NX_DSTAMP(7);
  if (threadIdx.x == 0)  // (every other workgroup has arrived: nothing counts after this)
    __hip_atomic_store(da.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (keep) dir_chain_asm<W, CPL>(pa, da, c0 + (int)threadIdx.x / W, c0 + (int)threadIdx.x / W < c1, L);
  stores();
}

// Factored coefficients from this solve's D (after the start application).
__global__ void k_pc_factor(PcArgs pa, int n_dc, int n_slots) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_dc) {
    const int lo = pa.dc_lo[i];
    pa.dc_kappa[i] = lo >= 0 ? 1.0 / pa.chain_T[pa.slot_dc[i]] / pa.slot_D[lo] : 0.0;
  }
  if (i < n_slots) pa.slot_invD[i] = 1.0 / pa.slot_D[i];
}

// Several ranks, dense top: root (coarse index) of every top slot and the response w_t of
// t to a unit value at its coarse root (w = prod of g_up / D along the path). Once per solve.
__global__ __launch_bounds__(kTopThreads) void k_pc_wroot(PcArgs pa) {
  const int ts0 = pa.top_lvl_off[0];
  for (int lv = 0; lv < pa.n_top_lvl; ++lv) {
    for (int t = pa.top_lvl_off[lv] + threadIdx.x; t < pa.top_lvl_off[lv + 1]; t += kTopThreads) {
      const int p = pa.slot_parent[t];
      if (p < ts0) {
        const int c = pa.slot_cidx[t];
        pa.top_rootc[t - ts0] = c;
        pa.top_w[t - ts0] = c >= 0 ? 1.0 : 0.0;
      } else {
        pa.top_rootc[t - ts0] = pa.top_rootc[p - ts0];
        pa.top_w[t - ts0] =
            pa.top_w[p - ts0] / pa.chain_T[pa.slot_pchain[t]] / pa.slot_D[t];
      }
    }
    __syncthreads();
  }
}

// Several ranks, dense top, every iteration: a = the summed top inputs, then this rank's
// coarse partials [D | J | G] (D fixed by the assembly, J = KJ[root,:] a, coarse chains).
// One workgroup of kTopThreads threads (its own kernel, or the up sweep's last workgroup).
__device__ void pc_cpart_body(const PcArgs& pa, double* sA);

__global__ __launch_bounds__(kTopThreads) void k_pc_cpart(PcArgs pa, const MrState* __restrict__ st,
                                                          int mode) {
  __shared__ double sA[kCapT];
  if (mode == 0 && st->done) return;
  pc_cpart_body(pa, sA);
}

// The fused k_pc_cpart: the last workgroup of the up sweep to finish (atomic ticket; every
// workgroup fences its writes first, the last one fences before reading) runs the body and
// resets the ticket for the next launch.
__device__ void pc_cpart_last(const PcArgs& pa, double* sA) {
  __shared__ int sLast;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    sLast = atomicAdd(pa.ticket, 1) == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!sLast) return;
  __threadfence();
  pc_cpart_body(pa, sA);
  if (threadIdx.x == 0) *pa.ticket = 0;
}

__device__ void pc_cpart_body(const PcArgs& pa, double* sA) {
  // the coarse roots among the top slots, found by all threads at once (one round trip)
  // and listed in LDS: the waves then only visit those (any order: each writes its own
  // coarse slot)
  __shared__ int sRoot[kCapT], sRootC[kCapT];
  __shared__ int sNr;
  if (threadIdx.x == 0) sNr = 0;
  __syncthreads();
  const int ts0 = pa.top_lvl_off[0], nt = pa.n_top, nC = pa.n_coarse;
  for (int sl = threadIdx.x; sl < nt; sl += kTopThreads) {
    const int c = pa.slot_cidx[ts0 + sl];
    const int par = pa.slot_parent[ts0 + sl];
    double a = 0.0;
    for (int i = pa.top_uoff[sl]; i < pa.top_uoff[sl + 1]; ++i) a += pa.u[i];
    sA[sl] = a;
    pa.atop[sl] = a;
    if (c >= 0 && par < ts0) {
      const int q = atomicAdd(&sNr, 1);
      sRoot[q] = sl;
      sRootC[q] = c;
    }
  }
  for (int i = threadIdx.x; i < 3 * nC; i += kTopThreads) pa.cbuf[i] = 0.0;
  __syncthreads();
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  for (int q = wv; q < sNr; q += kTopThreads / 64) {  // one wave per coarse root
    const int r = sRoot[q], c = sRootC[q];
    const double* __restrict__ k = pa.KJ + (int64_t)r * nt;
    double acc = 0.0;
    for (int sl = ln; sl < nt; sl += 64) acc += k[sl] * sA[sl];
    acc = wave_sum(acc);
    if (ln == 0) {
      pa.cbuf[c] = pa.slot_D[ts0 + r];
      pa.cbuf[nC + c] = acc;
    }
  }
  __syncthreads();
  const int ncc = pa.n_cc;
  if (ncc > 0 && nC <= kCapCoarseLds && ncc <= kCapCoarseLds) {
    // chains joining two coarse junctions: their data gathered in parallel, then summed
    // in LDS by one thread in the fixed order (same bits as summing in global memory,
    // without a dependent global round trip per chain)
    __shared__ double sCb[3 * kCapCoarseLds], sQg[kCapCoarseLds], sQt[kCapCoarseLds],
        sQb[kCapCoarseLds];
    __shared__ int sQi[kCapCoarseLds], sQo[kCapCoarseLds];
    for (int i = threadIdx.x; i < 3 * nC; i += kTopThreads) sCb[i] = pa.cbuf[i];
    for (int i = threadIdx.x; i < ncc; i += kTopThreads) {
      const int c = pa.cc_chain[i];
      sQg[i] = 1.0 / pa.chain_T[c];
      sQt[i] = pa.chain_It[c];
      sQb[i] = pa.chain_Ib[c];
      sQi[i] = pa.cc_top[i];
      sQo[i] = pa.cc_bot[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int i = 0; i < ncc; ++i) {
        const int t = sQi[i], b = sQo[i];
        const double g = sQg[i];
        sCb[t] += g;
        sCb[b] += g;
        sCb[nC + t] += sQt[i];
        sCb[nC + b] += sQb[i];
        sCb[2 * nC + b] = g;
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * nC; i += kTopThreads) pa.cbuf[i] = sCb[i];
  } else if (threadIdx.x == 0) {  // (large coarse sets) serial in global memory
    for (int i = 0; i < ncc; ++i) {
      const int c = pa.cc_chain[i], t = pa.cc_top[i], b = pa.cc_bot[i];
      const double g = 1.0 / pa.chain_T[c];
      pa.cbuf[t] += g;
      pa.cbuf[b] += g;
      pa.cbuf[nC + t] += pa.chain_It[c];
      pa.cbuf[nC + b] += pa.chain_Ib[c];
      pa.cbuf[2 * nC + b] = g;
    }
  }
}

// Dense top: column s of G = response of the top part to a unit J at top slot s (J up the
// ancestors with kappa = g_up / D, then the root-to-leaf back-substitution). One wave per
// column; once per solve (D is fixed by the assembly).
__device__ void pc_gbuild_column(const PcArgs& pa, int s);

__global__ __launch_bounds__(64) void k_pc_gbuild(PcArgs pa) { pc_gbuild_column(pa, blockIdx.x); }

// Single-rank head graph with the global-memory preconditioner kernels, once per solve:
// the factored coefficients (k_pc_factor), G's columns (k_pc_gbuild, n_gcols = n_top or
// 0) and optionally a copy r2 = b (n > 0). (The LDS path does this in k_pc_down_lds.)
__global__ __launch_bounds__(64) void k_pc_prep(PcArgs pa, int n_dc, int n_slots, int n_gcols,
                                                const double* __restrict__ b,
                                                double* __restrict__ r2, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 64;
  const int64_t i0 = (int64_t)blockIdx.x * 64 + threadIdx.x;
  for (int64_t i = i0; i < n; i += stride) r2[i] = b[i];
  for (int64_t i = i0; i < n_dc || i < n_slots; i += stride) {
    if (i < n_dc) {
      const int lo = pa.dc_lo[i];
      pa.dc_kappa[i] = lo >= 0 ? 1.0 / pa.chain_T[pa.slot_dc[i]] / pa.slot_D[lo] : 0.0;
    }
    if (i < n_slots) pa.slot_invD[i] = 1.0 / pa.slot_D[i];
  }
  if ((int)blockIdx.x < n_gcols) pc_gbuild_column(pa, blockIdx.x);
}

__device__ void pc_gbuild_column(const PcArgs& pa, int s) {
  __shared__ double sJ[kCapT], sZ[kCapT];
  const int nt = pa.n_top, ts0 = pa.top_lvl_off[0];
  for (int i = threadIdx.x; i < nt; i += 64) sJ[i] = 0.0;
  __syncthreads();
  const bool cd = pa.KJ != nullptr;  // several ranks: coarse roots are Dirichlet nodes
  if (threadIdx.x == 0) {
    double J = 1.0;
    int t = ts0 + s;
    sJ[s] = 1.0;
    for (int p = pa.slot_parent[t]; p >= ts0; t = p, p = pa.slot_parent[t]) {
      J = J / pa.chain_T[pa.slot_pchain[t]] / pa.slot_D[t];
      sJ[p - ts0] = J;
    }
    if (cd) {  // t is the root: its row of KJ for every root, this column
      for (int r = 0; r < nt; ++r) pa.KJ[(int64_t)r * nt + s] = 0.0;
      if (pa.slot_cidx[t] >= 0) pa.KJ[(int64_t)(t - ts0) * nt + s] = J;
    }
  }
  __syncthreads();
  for (int lv = 0; lv < pa.n_top_lvl; ++lv) {
    for (int u = pa.top_lvl_off[lv] + threadIdx.x; u < pa.top_lvl_off[lv + 1]; u += 64) {
      const int p = pa.slot_parent[u];
      double num = sJ[u - ts0];
      if (p >= ts0) num += sZ[p - ts0] / pa.chain_T[pa.slot_pchain[u]];
      sZ[u - ts0] = (cd && p < ts0 && pa.slot_cidx[u] >= 0) ? 0.0 : num / pa.slot_D[u];
    }
    __syncthreads();
  }
  for (int t = threadIdx.x; t < nt; t += 64) pa.G[(int64_t)t * nt + s] = sZ[t];
}

// Start application (k_pc_down_lds, mode 1; several ranks: fused mode): the factored
// coefficients and the columns s0, s0 + step, ... of G (same arithmetic as k_pc_factor /
// pc_gbuild_column), with the top part's parents, chain resistances, D and coarse indices
// staged in LDS once; several ranks also the KJ columns and, in workgroup 0, the roots and
// weights of k_pc_wroot. D is final here: the start's up and top (and coarse) kernels wrote it.
template <int BS>
__device__ void pc_prep_in_block(const PcArgs& pa, bool gcols, double* sJ, double* sZ, int* sPar,
                                 double* sTp, double* sDt, int* sCid) {
  if (pa.dc_kappa) {
    const int64_t stride = (int64_t)gridDim.x * BS;
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < pa.n_dc_all || i < pa.n_slots_all;
         i += stride) {
      if (i < pa.n_dc_all) {
        const int lo = pa.dc_lo[i];
        pa.dc_kappa[i] = lo >= 0 ? 1.0 / pa.chain_T[pa.slot_dc[i]] / pa.slot_D[lo] : 0.0;
      }
      if (i < pa.n_slots_all) pa.slot_invD[i] = 1.0 / pa.slot_D[i];
    }
  }
  if (!gcols || (int)blockIdx.x >= pa.n_top) return;  // block-uniform
  const int nt = pa.n_top, ts0 = pa.top_lvl_off[0];
  const bool cd = pa.KJ != nullptr;  // several ranks: coarse roots are Dirichlet nodes
  for (int u = threadIdx.x; u < nt; u += BS) {
    const int p = pa.slot_parent[ts0 + u];
    sPar[u] = p >= ts0 ? p - ts0 : -1;
    const int pc = pa.slot_pchain[ts0 + u];
    sTp[u] = pc >= 0 ? pa.chain_T[pc] : 1.0;
    sDt[u] = pa.slot_D[ts0 + u];
    sCid[u] = cd ? pa.slot_cidx[ts0 + u] : -1;
  }
  __syncthreads();
  for (int s = blockIdx.x; s < nt; s += gridDim.x) {
    for (int i = threadIdx.x; i < nt; i += BS) {
      sJ[i] = 0.0;
      if (cd) pa.KJ[(int64_t)i * nt + s] = 0.0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double J = 1.0;
      sJ[s] = 1.0;
      int t = s;
      for (int p = sPar[s]; p >= 0; t = p, p = sPar[t]) {
        J = J / sTp[t] / sDt[t];
        sJ[p] = J;
      }
      if (cd && sCid[t] >= 0) pa.KJ[(int64_t)t * nt + s] = J;  // t is the root
    }
    __syncthreads();
    for (int lv = 0; lv < pa.n_top_lvl; ++lv) {
      const int a = pa.top_lvl_off[lv] - ts0, b = pa.top_lvl_off[lv + 1] - ts0;
      for (int u = a + threadIdx.x; u < b; u += BS) {
        const int p = sPar[u];
        double num = sJ[u];
        if (p >= 0) num += sZ[p] / sTp[u];
        sZ[u] = (cd && p < 0 && sCid[u] >= 0) ? 0.0 : num / sDt[u];
      }
      __syncthreads();
    }
    for (int t = threadIdx.x; t < nt; t += BS) pa.G[(int64_t)t * nt + s] = sZ[t];
    __syncthreads();
  }
  if (cd && blockIdx.x == 0) {  // k_pc_wroot: coarse root and weight of every top slot
    for (int lv = 0; lv < pa.n_top_lvl; ++lv) {
      const int a = pa.top_lvl_off[lv] - ts0, b = pa.top_lvl_off[lv + 1] - ts0;
      for (int t = a + threadIdx.x; t < b; t += BS) {
        const int p = sPar[t];
        if (p < 0) {
          const int c = sCid[t];
          sCid[t] = c;  // own root index (already there)
          sJ[t] = c >= 0 ? 1.0 : 0.0;
        } else {
          sCid[t] = sCid[p];
          sJ[t] = sJ[p] / sTp[t] / sDt[t];
        }
      }
      __syncthreads();
    }
    for (int t = threadIdx.x; t < nt; t += BS) {
      pa.top_rootc[t] = sCid[t];
      pa.top_w[t] = sJ[t];
    }
  }
}

// Second half of the top part with several ranks: solve the coarse forest from the
// all-reduced [D | J | G] (every rank identically), then back-substitute the top part --
// coarse slots take their coarse value -- and the partial r.z of the top slots.
constexpr int kCapCoarse = 2048;

// Coarse forest solve (redundant on every rank: same inputs, same order, same bits) and the
// back-substitution of this rank's top part from the exact coarse values. Latency-bound, one
// workgroup: the top part's per-solve inputs (J, D, the parent chain's T) and structure are
// loaded into registers before the coarse solve (one slot per thread, the host caps the top
// part at 1024) and staged in LDS after it, and a small coarse forest is solved from LDS
// (pc_coarse_lds), so the level sweeps touch no global memory (8-rank depth-17 rehearsal:
// 31.8 us per launch with per-level global loads).
__global__ __launch_bounds__(kTopThreads) void k_pc_coarse(PcArgs pa, double* __restrict__ y,
                                                           const double* __restrict__ r2,
                                                           double* __restrict__ z,
                                                           MrState* __restrict__ st,
                                                           double* __restrict__ partB, int mode) {
  __shared__ double sD[kCapCoarse], sJ[kCapCoarse], sZ[kCapCoarse];
  __shared__ int sTp[kTopThreads], sTl[kTopThreads];  // top slot: parent (local) or -2 - coarse index; lambda
  __shared__ int sTlv[kMaxTopLvl + 1];  // the top levels' slot offsets
  if (mode == 0 && st->done) return;
  // linear form: alpha arrived with the coarse partials; the Lanczos step is completed here
  double c2 = 0.0;
  const bool lin = pa.lin && mode == 0;
  if (lin) {
    const double alfa = pa.xalpha[0];
    c2 = alfa / st->beta;
    __syncthreads();  // every thread has read st->beta before thread 0 updates st
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->alfa = alfa;
      st->nb += 1;
    }
  }
  const int nC = pa.n_coarse;
  const bool backsub = !(pa.mdense && mode == 0);
  const int ntl = pa.n_top_lvl;
  const int ts0 = ntl > 0 ? pa.top_lvl_off[0] : 0;
  const int nt = ntl > 0 ? pa.top_lvl_off[ntl] - ts0 : 0;
  const bool staged = backsub && nt <= kTopThreads;
  // this thread's top slot, loaded before the coarse solve (hides the global round trips)
  const int sl0 = threadIdx.x;
  int t_k = -1, t_lam = 0, t_par = -1;
  double t_J = 0.0, t_D = 1.0, t_T = 1.0;
  // the top levels' offsets (thread <= ntl), staged in LDS after the coarse solve
  const int t_lvo = staged && (int)threadIdx.x <= ntl && ntl <= kMaxTopLvl ? pa.top_lvl_off[threadIdx.x] : 0;
  double t_y = 0.0;  // y at this slot's multiplier (finish)
  if (staged && sl0 < nt) {
    const int j = ts0 + sl0;
    t_k = pa.slot_cidx[j];
    t_lam = pa.slot_lam[j];
    t_y = y[t_lam];
    if (t_k < 0) {
      t_par = pa.slot_parent[j];
      t_J = pa.slot_J[j];
      t_D = pa.slot_D[j];
      if (t_par >= 0) t_T = pa.chain_T[pa.slot_pchain[j]];
    }
  }
  const double* __restrict__ G = pa.cbuf + 2 * nC;
  if (nC <= kCapCoarseLds) {
    pc_coarse_lds(pa, sD, sJ, sZ);
  } else {
    for (int i = threadIdx.x; i < nC; i += kTopThreads) {
      sD[i] = pa.cbuf[i];
      sJ[i] = pa.cbuf[nC + i];
    }
    __syncthreads();
    for (int lv = pa.n_clvl - 1; lv >= 0; --lv) {  // deepest level first
      for (int j = pa.c_lvl_off[lv] + threadIdx.x; j < pa.c_lvl_off[lv + 1]; j += kTopThreads) {
        double D = sD[j], J = sJ[j];
        for (int i = pa.c_child_off[j]; i < pa.c_child_off[j + 1]; ++i) {
          const int k = pa.c_child[i];
          const double g = G[k], Dk = sD[k];
          D -= g * g / Dk;
          J += g * sJ[k] / Dk;
        }
        sD[j] = D;
        sJ[j] = J;
      }
      __syncthreads();
    }
    for (int lv = 0; lv < pa.n_clvl; ++lv) {  // root level first
      for (int j = pa.c_lvl_off[lv] + threadIdx.x; j < pa.c_lvl_off[lv + 1]; j += kTopThreads) {
        const int p = pa.c_parent[j];
        sZ[j] = (sJ[j] + (p >= 0 ? G[j] * sZ[p] : 0.0)) / sD[j];
      }
      __syncthreads();
    }
  }
  if (!backsub) {  // the down kernels evaluate the top part (dense rows)
    for (int j = threadIdx.x; j < nC; j += kTopThreads) pa.zc[j] = sZ[j];
    if (threadIdx.x == 0) partB[pa.n_jobs] = 0.0;
    return;
  }
  double part = 0.0;
  auto finish = [&](int j, int lam, double zj, bool pre = false) {
    pa.slot_z[j] = zj;
    double yl = pre ? t_y : y[lam];
    if (lin) {  // ghost slots: y = r2 = 0 and the halo overwrites z
      zj -= c2 * z[lam];
      yl -= c2 * r2[lam];
      y[lam] = yl;
    }
    if (mode == kModeDirect && pa.accum)
      z[lam] += zj;
    else
      z[lam] = zj;
    part += yl * zj;
  };
  if (staged) {  // sD / sJ are free now: J, D | T, z of the top slots
    double* sTJ = sD;
    double* sTD = sD + kTopThreads;
    double* sTT = sJ;
    double* sTZ = sJ + kTopThreads;
    if (sl0 < nt) {
      sTJ[sl0] = t_J;
      sTD[sl0] = t_D;
      sTT[sl0] = t_T;
      sTp[sl0] = t_k >= 0 ? -2 - t_k : (t_par >= 0 ? t_par - ts0 : -1);
      sTl[sl0] = t_lam;
    }
    if ((int)threadIdx.x <= ntl && ntl <= kMaxTopLvl) sTlv[threadIdx.x] = t_lvo;
    __syncthreads();
    if (ntl <= kMaxTopLvl) {  // thread = slot: its level and inputs in registers
      int mylv = -1;
      if (sl0 < nt)
        for (int q = 0; q < ntl; ++q)
          if (ts0 + sl0 >= sTlv[q] && ts0 + sl0 < sTlv[q + 1]) mylv = q;
      const int p = t_k >= 0 ? -2 - t_k : (t_par >= 0 ? t_par - ts0 : -1);
      for (int lv = 0; lv < ntl; ++lv) {
        if (mylv == lv) {
          double zj;
          if (p <= -2) {
            zj = sZ[-2 - p];
          } else {
            double num = t_J;
            if (p >= 0) num += sTZ[p] / t_T;
            zj = num / t_D;
          }
          sTZ[sl0] = zj;
          finish(ts0 + sl0, t_lam, zj, true);
        }
        __syncthreads();
      }
    } else
    for (int lv = 0; lv < ntl; ++lv) {
      for (int j = pa.top_lvl_off[lv] + threadIdx.x; j < pa.top_lvl_off[lv + 1]; j += kTopThreads) {
        const int sl = j - ts0;
        const int p = sTp[sl];
        double zj;
        if (p <= -2) {
          zj = sZ[-2 - p];
        } else {
          double num = sTJ[sl];
          if (p >= 0) num += sTZ[p] / sTT[sl];
          zj = num / sTD[sl];
        }
        sTZ[sl] = zj;
        finish(j, sTl[sl], zj);
      }
      __syncthreads();
    }
  } else {
    for (int lv = 0; lv < ntl; ++lv) {
      for (int j = pa.top_lvl_off[lv] + threadIdx.x; j < pa.top_lvl_off[lv + 1]; j += kTopThreads) {
        const int k = pa.slot_cidx[j];
        double zj;
        if (k >= 0) {
          zj = sZ[k];
        } else {
          const int p = pa.slot_parent[j];
          double num = pa.slot_J[j];
          if (p >= 0) num += pa.slot_z[p] / pa.chain_T[pa.slot_pchain[j]];
          zj = num / pa.slot_D[j];
        }
        finish(j, pa.slot_lam[j], zj);
      }
      __syncthreads();
    }
  }
  block_sum_store_n<kTopThreads>(part, partB + pa.n_jobs);
}

__global__ void k_pack(const double* __restrict__ x, const int* __restrict__ idx, int n,
                       double* __restrict__ buf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) buf[i] = x[idx[i]];
}

// Solution in the reference's block order (nx_get_solution_blocks): out[i] = x[idx[i]],
// idx = the [flux colour 0 .. M-1 | pressure | multiplier] permutation of the owned rows.
__global__ __launch_bounds__(kBlock) void k_gather_out(const double* __restrict__ x,
                                                       const int* __restrict__ idx, int64_t n,
                                                       double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = x[idx[i]];
}

// ---- Direct solve (nx_set_solver(h, 1)): block LU of the symmetric system A = [[M, K],
// [K^T, 0]] (flux rows q; pressure cells and multipliers s), whose Schur complement
// S = K^T M^{-1} K is exactly what the tree preconditioner inverts (P = blockdiag(M, S);
// precond.py): y = M^{-1} b_q, x_s = S^{-1} (K^T y - b_s), x_q = M^{-1} (b_q - K x_s), all
// inside the LDS sweeps' mode 3 (kModeDirect; one rank: k_dir_step), then the true residual.
// This is the reference's default ksp_type=preonly + pc_type=lu (a direct factorisation,
// solver.py:58-65) specialised to the network's tree structure (graphs with cycles: the
// Woodbury correction of the cycle chains, k_cyc_*).


// Several ranks, fused check: this rank's ||r||^2, ||b||^2 (the down sweeps' partials in job
// order, then its owned rows no job could form -- the top part's and the cut junctions'
// multiplier rows, after the halo of x -- from the CSR, r stored) -> out[0], out[1].
__global__ __launch_bounds__(kReduceThreads) void k_dir_reduce2_fr(
    const double* __restrict__ rpart, int nj, const int* __restrict__ left, int nleft, Csr A,
    const double* __restrict__ x, const double* __restrict__ b, double* __restrict__ rres,
    double* __restrict__ bbst, int refine, double* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ double s_r[kReduceThreads / 64], s_b[kReduceThreads / 64];
  double rr = 0.0, bb = 0.0;
  for (int i = threadIdx.x; i < nj; i += kReduceThreads) {
    rr += rpart[i];
    bb += rpart[nj + i];
  }
  for (int i = threadIdx.x; i < nleft; i += kReduceThreads) {
    const int row = left[i];
    double acc = 0.0;
    for (int k = A.rowptr[row]; k < A.rowptr[row + 1]; ++k) acc += A.val[k] * x[A.col[k]];
    const double bv = b[row];
    const double rv = bv - acc;
    rres[row] = rv;
    rr += rv * rv;
    bb += bv * bv;
  }
  rr = wave_sum(rr);
  bb = wave_sum(bb);
  if ((threadIdx.x & 63) == 0) {
    s_r[threadIdx.x >> 6] = rr;
    s_b[threadIdx.x >> 6] = bb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    rr = 0.0;
    bb = 0.0;
    for (int w = 0; w < kReduceThreads / 64; ++w) {
      rr += s_r[w];
      bb += s_b[w];
    }
    if (refine)
      bb = bbst[0];
    else
      bbst[0] = bb;
    out[0] = rr;
    out[1] = bb;
  }
}

// Several ranks, fused check with the cut rows (nx_set_cut): as k_dir_reduce2_fr, but an
// owned cut bifurcation's row is summed over its owned columns only and left as a partial
// in out[2 + k], and this rank's share of every cut row it does not own (its flux ends
// there, -(+-1) x_q in a fixed order) goes to out[2 + k] too; out[0], out[1] exclude the
// cut rows' r^2 (k_dir_publish_cut adds them after the all-reduce of out).
__global__ __launch_bounds__(kReduceThreads) void k_dir_reduce_cut(
    const double* __restrict__ rpart, int nj, const int* __restrict__ left,
    const int* __restrict__ left_k, int nleft, Csr A, double* __restrict__ x,
    const double* __restrict__ b, double* __restrict__ rres, double* __restrict__ bbst,
    int refine, int K, const int* __restrict__ cut_own, const int* __restrict__ gk_off,
    const int* __restrict__ gk_row, const double* __restrict__ gk_coef,
    double* __restrict__ out, const int* __restrict__ top_lam,
    const double* __restrict__ top_z, int ntop) {
#pragma clang fp contract(off)
  __shared__ double s_r[kReduceThreads / 64], s_b[kReduceThreads / 64];
  // coarsedown: the top part's values (every down workgroup solved them, workgroup 0's copy
  // in slot_z) into x; the rows below read flux values only
  for (int i = threadIdx.x; i < ntop; i += kReduceThreads) {
    const int lam = top_lam[i];
    if (refine)
      x[lam] += top_z[i];
    else
      x[lam] = top_z[i];
  }
  double rr = 0.0, bb = 0.0;
  for (int i = threadIdx.x; i < nj; i += kReduceThreads) {
    rr += rpart[i];
    bb += rpart[nj + i];
  }
  for (int i = threadIdx.x; i < nleft; i += kReduceThreads) {
    const int row = left[i];
    double acc = 0.0;
    for (int k = A.rowptr[row]; k < A.rowptr[row + 1]; ++k) {
      const int c = A.col[k];
      if (c < A.n_rows) acc += A.val[k] * x[c];  // ghost columns: their owners' share
    }
    const double bv = b[row];
    const double rv = bv - acc;
    bb += bv * bv;
    const int kc = left_k[i];
    if (kc >= 0) {
      out[2 + kc] = rv;
    } else {
      rres[row] = rv;
      rr += rv * rv;
    }
  }
  // cut index k on thread kReduceThreads - 1 - k: beside the left rows' threads, not after
  for (int k = kReduceThreads - 1 - (int)threadIdx.x; k >= 0 && k < K; k += kReduceThreads) {
    if (cut_own[k] >= 0) continue;  // written above
    double sh = 0.0;
    for (int e = gk_off[k]; e < gk_off[k + 1]; ++e) sh -= gk_coef[e] * x[gk_row[e]];
    out[2 + k] = sh;
  }
  rr = wave_sum(rr);
  bb = wave_sum(bb);
  if ((threadIdx.x & 63) == 0) {
    s_r[threadIdx.x >> 6] = rr;
    s_b[threadIdx.x >> 6] = bb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    rr = 0.0;
    bb = 0.0;
    for (int w = 0; w < kReduceThreads / 64; ++w) {
      rr += s_r[w];
      bb += s_b[w];
    }
    if (refine)
      bb = bbst[0];
    else
      bbst[0] = bb;
    out[0] = rr;
    out[1] = bb;
  }
}

// After the all-reduce of [rr, bb, r_cut]: the cut rows' r^2 added in index order (every
// rank the same bits), the owned ones' r stored for a refinement step, the state published.
__global__ void k_dir_publish_cut(const double* __restrict__ rb, int K,
                                  const int* __restrict__ cut_own, double* __restrict__ rres,
                                  double rtol, int* seq, MrState* mirror) {
#pragma clang fp contract(off)
  if (threadIdx.x != 0) return;
  double rr = rb[0];
  for (int k = 0; k < K; ++k) {
    const double r = rb[2 + k];
    rr += r * r;
    if (cut_own[k] >= 0) rres[cut_own[k]] = r;
  }
  const double bb = rb[1];
  MrState s{};
  s.beta1 = sqrt(bb);
  s.relres = bb > 0.0 ? sqrt(rr / bb) : sqrt(rr);
  s.rtol = rtol;
  s.it = 1;
  s.done = 1;
  s.converged = s.relres <= rtol ? 1 : 0;
  MrInit ini{};
  ini.seq = seq;
  ini.mirror = mirror;
  mr_publish(s, ini);
}

__global__ void k_dir_publish_red(const double* __restrict__ rb, double rtol, int* seq,
                                  MrState* mirror) {
  if (threadIdx.x != 0) return;
  const double rr = rb[0], bb = rb[1];
  MrState s{};
  s.beta1 = sqrt(bb);
  s.relres = bb > 0.0 ? sqrt(rr / bb) : sqrt(rr);
  s.rtol = rtol;
  s.it = 1;
  s.done = 1;
  s.converged = s.relres <= rtol ? 1 : 0;
  MrInit ini{};
  ini.seq = seq;
  ini.mirror = mirror;
  mr_publish(s, ini);
}

// ---- graphs with cycles (one rank, nx_set_cycles). The tree solve inverts A_g = A minus
// the couplings a = A[q, lam] = A[lam, q] of the m/2 cycle-closing chains' grounded ends
// (U = the unit columns of those rows, A = A_g + U C U^T, C = blocks [[0, a], [a, 0]]), so
//   A^{-1} b = x_g - Z Cinv U^T x_g,  x_g = A_g^{-1} b,  Z = A_g^{-1} U,
//   Cinv = (C^{-1} + U^T Z)^{-1}                                   (Woodbury),
// with Z (m columns) and Cinv built once per assembled matrix (cyc_build).
// cycle-closing chains (m = 2 kMaxCyc columns; round 6: the capacitance matrix is inverted on
// the device, cyc_invert, and the correction's kernels hold U^T x in dynamic LDS -- was 128)
constexpr int kMaxCyc = 2048;

// The m x m matrix U^T Z and the couplings a (row q of the CSR, column lam).
__global__ __launch_bounds__(256) void k_cyc_cap(Csr A, const double* __restrict__ Z, int64_t ldz,
                                                 const int* __restrict__ rows, int m,
                                                 double* __restrict__ cap, double* __restrict__ acoef) {
  for (int i = threadIdx.x; i < m * m; i += 256) {
    const int r = i / m, c = i % m;
    cap[i] = Z[(int64_t)c * ldz + rows[r]];
  }
  for (int k = threadIdx.x; 2 * k < m; k += 256) {
    const int q = rows[2 * k], lam = rows[2 * k + 1];
    double a = 0.0;
    for (int p = A.rowptr[q]; p < A.rowptr[q + 1]; ++p)
      if (A.col[p] == lam) a = A.val[p];
    acoef[k] = a;
  }
}

// w = Cinv (U^T x - prev) (prev: U^T x before a refinement pass added its correction, or
// null); save: U^T x is stored there instead (before a refinement pass). One workgroup.
// Cinv is stored transposed (cinvT[j m + i] = Cinv[i][j]: a row per thread, coalesced); one
// row of w per thread over ceil(m / 256) blocks (cyc_w_launch), U^T x in dynamic LDS (m doubles).
__global__ __launch_bounds__(256) void k_cyc_w(const double* __restrict__ x, const int* __restrict__ rows,
                                               int m, const double* __restrict__ cinvT,
                                               const double* __restrict__ prev, double* __restrict__ w,
                                               double* __restrict__ save) {
  extern __shared__ double g[];
  for (int i = threadIdx.x; i < m; i += 256) {
    const double v = x[rows[i]];
    if (save && blockIdx.x == 0) save[i] = v;
    g[i] = prev ? v - prev[i] : v;
  }
  if (save) return;
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= m) return;
  double s = 0.0;
  for (int j = 0; j < m; ++j) s += cinvT[(int64_t)j * m + i] * g[j];
  w[i] = s;
}

// x -= Z w, one row per thread (the m columns in order).
__global__ __launch_bounds__(kBlock) void k_cyc_fix(double* __restrict__ x, const double* __restrict__ Z,
                                                    int64_t ldz, const double* __restrict__ w, int m,
                                                    int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int j = 0; j < m; ++j) s += Z[(int64_t)j * ldz + i] * w[j];
  x[i] -= s;
}

// b = e_row: the right-hand side of one column of Z (b zeroed before; several ranks: only
// the row's owner sets it, rows[j] < 0 elsewhere)
__global__ void k_cyc_unit(double* __restrict__ b, const int* __restrict__ rows, int j) {
  if (rows[j] >= 0) b[rows[j]] = 1.0;
}

// ---- graphs with cycles, several ranks (nx_set_cycles_team): the same Woodbury correction
// with U's m rows spread over the ranks (a cycle chain's flux end lives with the chain, its
// multiplier row with the bifurcation's owner). own[i]: this rank's row of U's column i,
// or -1. Per assembled matrix every rank's share of U^T Z and of the couplings is summed over
// the ranks (one all-reduce); per solve U^T x is (one all-reduce of m).

// u_i = x[own_i] on this rank's rows, 0 elsewhere (summed over the ranks next)
__global__ __launch_bounds__(256) void k_cyc_gather(const double* __restrict__ x,
                                                    const int* __restrict__ own, int m,
                                                    double* __restrict__ u) {
  for (int i = threadIdx.x; i < m; i += 256) u[i] = own[i] >= 0 ? x[own[i]] : 0.0;
}

// This rank's share of U^T Z (rows of U it owns) and of the couplings a (the cycle chains it
// holds: row q, column lam -- maybe a ghost column -- of its CSR).
__global__ __launch_bounds__(256) void k_cyc_cap_team(Csr A, const double* __restrict__ Z, int64_t ldz,
                                                      const int* __restrict__ own, int m,
                                                      const int* __restrict__ qloc,
                                                      const int* __restrict__ lcol,
                                                      double* __restrict__ cap,
                                                      double* __restrict__ acoef) {
  for (int i = threadIdx.x; i < m * m; i += 256) {
    const int r = i / m, c = i % m;
    cap[i] = own[r] >= 0 ? Z[(int64_t)c * ldz + own[r]] : 0.0;
  }
  for (int k = threadIdx.x; 2 * k < m; k += 256) {
    double a = 0.0;
    if (qloc[k] >= 0)
      for (int p = A.rowptr[qloc[k]]; p < A.rowptr[qloc[k] + 1]; ++p)
        if (A.col[p] == lcol[k]) a = A.val[p];
    acoef[k] = a;
  }
}

// w = Cinv (u - prev) from the summed u (prev: U^T x before a refinement pass, or null).
__global__ __launch_bounds__(256) void k_cyc_w_team(const double* __restrict__ u, int m,
                                                    const double* __restrict__ cinvT,
                                                    const double* __restrict__ prev,
                                                    double* __restrict__ w) {
  extern __shared__ double g[];
  for (int i = threadIdx.x; i < m; i += 256) g[i] = prev ? u[i] - prev[i] : u[i];
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= m) return;
  double s = 0.0;
  for (int j = 0; j < m; ++j) s += cinvT[(int64_t)j * m + i] * g[j];
  w[i] = s;
}

// ---- the capacitance matrix's inverse on the device (cyc_invert): Gauss-Jordan with partial
// pivoting on [A | I] (row-major, m x 2m), one column per pair of launches -- the pivot row
// found, swapped in and normalised by one workgroup, then every other row eliminated by a
// workgroup each -- the same operations in the same order on every rank (the same bits).
// A = U^T Z + C^{-1}: C^{-1} of the coupling blocks [[0, a], [a, 0]] is [[0, 1/a], [1/a, 0]].
__global__ __launch_bounds__(256) void k_gj_init(const double* __restrict__ cap, int m,
                                                 double* __restrict__ aug, int* __restrict__ bad) {
  const int64_t n = (int64_t)m * 2 * m;
  for (int64_t t = blockIdx.x * (int64_t)256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const int r = (int)(t / (2 * m)), c = (int)(t % (2 * m));
    double v;
    if (c < m) {
      v = cap[(int64_t)r * m + c];
      if ((r >> 1) == (c >> 1) && r != c) {  // the coupling pair's off-diagonal
        const double a = cap[(int64_t)m * m + (r >> 1)];
        if (a == 0.0) *bad = 1;  // (no coupling at a grounded end: cyc_invert fails)
        v += 1.0 / a;
      }
    } else {
      v = c - m == r ? 1.0 : 0.0;
    }
    aug[t] = v;
  }
}

__global__ __launch_bounds__(1024) void k_gj_pivot(double* __restrict__ aug, int m, int col,
                                                   int* __restrict__ bad) {
  __shared__ double sv[1024];
  __shared__ int si[1024];
  const int w = 2 * m;
  double best = -1.0;
  int bi = col;
  for (int r = col + threadIdx.x; r < m; r += 1024) {
    const double v = fabs(aug[(int64_t)r * w + col]);
    if (v > best) {  // (strictly: the first row of the largest magnitude in this thread)
      best = v;
      bi = r;
    }
  }
  sv[threadIdx.x] = best;
  si[threadIdx.x] = bi;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      const double a = sv[threadIdx.x], b = sv[threadIdx.x + o];
      const int ia = si[threadIdx.x], ib = si[threadIdx.x + o];
      if (b > a || (b == a && ib < ia)) {  // ties: the smaller row, as a serial scan
        sv[threadIdx.x] = b;
        si[threadIdx.x] = ib;
      }
    }
    __syncthreads();
  }
  const int p = si[0];
  if (!(sv[0] > 0.0)) {
    if (threadIdx.x == 0) *bad = 2;
    return;
  }
  if (p != col)
    for (int c = threadIdx.x; c < w; c += 1024) {
      const double t = aug[(int64_t)col * w + c];
      aug[(int64_t)col * w + c] = aug[(int64_t)p * w + c];
      aug[(int64_t)p * w + c] = t;
    }
  __syncthreads();
  const double d = 1.0 / aug[(int64_t)col * w + col];
  __syncthreads();  // (every thread holds the pivot before row col changes)
  for (int c = threadIdx.x; c < w; c += 1024) aug[(int64_t)col * w + c] *= d;
}

__global__ __launch_bounds__(256) void k_gj_elim(double* __restrict__ aug, int m, int col) {
  const int r = blockIdx.x;
  if (r == col) return;
  const int w = 2 * m;
  const double f = aug[(int64_t)r * w + col];
  if (f == 0.0) return;
  __syncthreads();  // (f read by every thread before column col of this row changes)
  const double* __restrict__ pr = aug + (int64_t)col * w;
  double* __restrict__ rr = aug + (int64_t)r * w;
  for (int c = threadIdx.x; c < w; c += 256) rr[c] -= f * pr[c];
}

// cinvT[j m + i] = inverse[i][j] (the right half of the reduced [I | A^{-1}])
__global__ __launch_bounds__(256) void k_gj_out(const double* __restrict__ aug, int m,
                                                double* __restrict__ cinvT) {
  const int64_t n = (int64_t)m * m;
  for (int64_t t = blockIdx.x * (int64_t)256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const int j = (int)(t / m), i = (int)(t % m);
    cinvT[t] = aug[(int64_t)i * 2 * m + m + j];
  }
}

// ||b - A x|| / ||b|| from k_residual's partials (fixed order), published like a MINRES
// state (it = 1, done) to the host-coherent mirror the host spins on.
__global__ __launch_bounds__(kReduceThreads) void k_dir_publish(const double* __restrict__ p,
                                                                int nblk, double rtol, int* seq,
                                                                MrState* mirror) {
  // both sums in one pass (fixed order: thread-strided, then waves, then thread 0)
  __shared__ double s_r[kReduceThreads / 64], s_b[kReduceThreads / 64];
  double rr = 0.0, bb = 0.0;
  for (int i = threadIdx.x; i < nblk; i += kReduceThreads) {
    rr += p[i];
    bb += p[nblk + i];
  }
  rr = wave_sum(rr);
  bb = wave_sum(bb);
  if ((threadIdx.x & 63) == 0) {
    s_r[threadIdx.x >> 6] = rr;
    s_b[threadIdx.x >> 6] = bb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    rr = 0.0;
    bb = 0.0;
    for (int w = 0; w < kReduceThreads / 64; ++w) {
      rr += s_r[w];
      bb += s_b[w];
    }
    MrState s{};
    s.beta1 = sqrt(bb);
    s.relres = bb > 0.0 ? sqrt(rr / bb) : sqrt(rr);
    s.rtol = rtol;
    s.it = 1;
    s.done = 1;
    s.converged = s.relres <= rtol ? 1 : 0;
    MrInit ini{};
    ini.seq = seq;
    ini.mirror = mirror;
    mr_publish(s, ini);
  }
}

// The fused check's publish step (pa.fres): the down sweeps' partials in job order, then the
// rows no job could form (multiplier rows of junctions whose chains span jobs -- the top
// part) from the CSR: r = b - A x, stored for a refinement step. ||b||^2 is that of the
// first pass (bbst); a refinement pass (refine = 1) reuses it.
__global__ __launch_bounds__(kReduceThreads) void k_dir_publish_fr(
    const double* __restrict__ rpart, int nj, const int* __restrict__ left, int nleft, Csr A,
    double* __restrict__ x, const double* __restrict__ b, double* __restrict__ rres,
    double* __restrict__ bbst, int refine, double rtol, int* seq, MrState* mirror,
    const int* __restrict__ top_lam, const double* __restrict__ top_z, int ntop) {
#pragma clang fp contract(off)
  // topdown: the top part's values (solved in every down workgroup, workgroup 0's copy in
  // slot_z) into x; the rows below read flux values only (multiplier rows)
  for (int i = threadIdx.x; i < ntop; i += kReduceThreads) {
    const int lam = top_lam[i];
    if (refine)
      x[lam] += top_z[i];
    else
      x[lam] = top_z[i];
  }
  __shared__ double s_r[kReduceThreads / 64], s_b[kReduceThreads / 64];
  double rr = 0.0, bb = 0.0;
  for (int i = threadIdx.x; i < nj; i += kReduceThreads) {
    rr += rpart[i];
    bb += rpart[nj + i];
  }
  for (int i = threadIdx.x; i < nleft; i += kReduceThreads) {
    const int row = left[i];
    double acc = 0.0;
    for (int k = A.rowptr[row]; k < A.rowptr[row + 1]; ++k) acc += A.val[k] * x[A.col[k]];
    const double bv = b[row];
    const double rv = bv - acc;
    rres[row] = rv;
    rr += rv * rv;
    bb += bv * bv;
  }
  rr = wave_sum(rr);
  bb = wave_sum(bb);
  if ((threadIdx.x & 63) == 0) {
    s_r[threadIdx.x >> 6] = rr;
    s_b[threadIdx.x >> 6] = bb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    rr = 0.0;
    bb = 0.0;
    for (int w = 0; w < kReduceThreads / 64; ++w) {
      rr += s_r[w];
      bb += s_b[w];
    }
    if (refine)
      bb = bbst[0];
    else
      bbst[0] = bb;
    MrState s{};
    s.beta1 = sqrt(bb);
    s.relres = bb > 0.0 ? sqrt(rr / bb) : sqrt(rr);
    s.rtol = rtol;
    s.it = 1;
    s.done = 1;
    s.converged = s.relres <= rtol ? 1 : 0;
    MrInit ini{};
    ini.seq = seq;
    ini.mirror = mirror;
    mr_publish(s, ini);
  }
}

// Halo pack + this rank's beta^2 (sum of the previous iteration's partials, block 0) into
// red[1] and its own slot of the gathered array: saves a reduction launch per iteration.
__global__ __launch_bounds__(kBlock) void k_pack_beta(const double* __restrict__ x,
                                                      const int* __restrict__ idx, int n,
                                                      double* __restrict__ buf,
                                                      const double* __restrict__ partB, int nB,
                                                      double* __restrict__ red1,
                                                      double* __restrict__ gath_self) {
  if (blockIdx.x == 0) {
    const double t = block_allsum(partB, nB);
    if (threadIdx.x == 0) {
      *red1 = t;
      *gath_self = t;
    }
  }
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) buf[i] = x[idx[i]];
}

// In-process group transport: sum n values over the ranks' buffers in rank order and
// store the total in every buffer (the RCCL all-reduce of a group on one device).
constexpr int kMaxGroup = 16;
struct GroupPtrs {
  double* p[kMaxGroup];
};

// dst[r][q] = src[q][0] for all ranks r, q (the group's point-to-point all-gather of one
// double per rank)
__global__ void k_group_gather(GroupPtrs src, GroupPtrs dst, int P) {
  const int i = threadIdx.x;
  if (i < P * P) dst.p[i / P][i % P] = src.p[i % P][0];
}

__global__ void k_group_sum(GroupPtrs g, int P, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int r = 0; r < P; ++r) s += g.p[r][i];
    for (int r = 0; r < P; ++r) g.p[r][i] = s;
  }
}

}  // namespace

// ======================================================================================
// Host side
// ======================================================================================

struct LeanGraphs {
  hipGraphExec_t head_exec = nullptr;
  hipGraph_t head_graph = nullptr;
  int head_len = 0;
  double head_rtol = 0.0;
  int head_maxit = 0;
  hipGraphExec_t lchunk_exec = nullptr;
  hipGraph_t lchunk_graph = nullptr;
  int lchunk_len = 0;
  double lchunk_rtol = 0.0;  // the direct solve's refinement graph (lchunk_len = -1)
  // direct tree solve (nx_set_solver(h, 1)): one graph per solve; the _asm one starts with
  // the deferred assembly of values and rhs
  hipGraphExec_t direct_exec = nullptr;
  hipGraph_t direct_graph = nullptr;
  int direct_len = 0;
  double direct_rtol = 0.0;
  hipGraphExec_t direct_asm_exec = nullptr;
  hipGraph_t direct_asm_graph = nullptr;
  int direct_asm_len = 0;
  double direct_asm_rtol = 0.0;
};

// the host transport (tests; its collectives are with the Team's): a shared-memory segment
// of a header (a barrier's counters) and one slot per rank
struct HcHdr {
  std::atomic<uint32_t> count;
  std::atomic<uint32_t> gen;
};
struct HostComm {
  int P = 0, rank = 0;
  size_t slot = 0, bytes = 0;
  unsigned char* base = nullptr;
  std::string name;
};

struct nx_network {
  int device = 0;
  hipStream_t stream = nullptr;
  int N = 0;
  int64_t E = 0, B = 0, n_edge_dofs = 0, n_own = 0, n_ghost = 0, n_col = 0;
  int64_t nnz_edges = 0, nnz_lm = 0, nnz = 0;
  int nblk = 0;  // blocks of kRowsPerBlock rows
  // topology / coefficients
  double* edge_x = nullptr;
  int* edge_lm = nullptr;
  int* edge_seg = nullptr;
  double* edge_R = nullptr;
  double* edge_bc = nullptr;
  double* edge_f = nullptr;  // per-edge source (nx_set_source), or null: f everywhere
  double* lm_val = nullptr;
  double* dq = nullptr;  // E*(N+1) lumped flux mass (preconditioner D block)
  double f = 0.0;
  bool have_coeffs = false, have_lhs = false, have_rhs = false;
  // CSR + rhs
  int* rowptr = nullptr;
  int* col = nullptr;
  double* val = nullptr;
  double* rhs = nullptr;
  // Krylov vectors
  double* vb[2] = {nullptr, nullptr};  // r1/r2, n_col each
  double* wb[2] = {nullptr, nullptr};  // w1/w2, n_own each
  double* x = nullptr;                 // n_col
  double* tmp = nullptr;               // n_col (host SpMV / residual)
  double* partials = nullptr;          // nblk (residual) >= nA + nB
  int nA = 1;                          // k_mr_a blocks (partials of alpha)
  int chunksA = kChunksADefault;       // 256-row chunks per k_mr_a block
  int nB = kBlocksBDefault;            // k_mr_b blocks (partials of beta^2)
  double* partA = nullptr;             // nA
  double* partB = nullptr;             // nB
  double* red = nullptr;               // 4 cross-rank reduction slots
  MrState* st = nullptr;               // 2 buffers (ping-pong)
  // tree Schur preconditioner (nx_set_preconditioner)
  bool pc = false;
  bool pc_lds = false;  // every job fits the LDS kernels' caps
  int pc_variant = 0;   // (W, CPL) instantiation
  // the fused step's (W, CPL) (k_dir_step / k_dir_xr / k_dir_xg): N <= 32 by 8 lanes so a
  // job's <= 128 chains run in ONE pass (phase 2 on phase 1's registers, no reloads): 2
  // cells per lane up to N = 16, 3 up to 24 (C4's N = 19), 4 up to 32 (register spills)
  int dstep_variant = 0;
  int pc_jobs = 0;
  int64_t pc_slots = 0;
  int64_t pc_ndc = 0;
  PcArgs pa{};
  std::vector<void*> pc_bufs;
  double* z = nullptr;  // P^{-1} r, n_col
  double* vv = nullptr; // Lanczos vector v, n_own
  double* vs = nullptr;   // stored Lanczos vectors v_1..v_kMaxV (kMaxV * n_own), or null
  double* hist = nullptr; // their rotations (4 * kMaxV)
  MrState* h_st = nullptr;             // pinned host mirror of both
  MrState* h_last = nullptr;           // host-coherent, mapped: the state published by the
  MrState* d_last = nullptr;           // last k_mr_a of a lean graph (mr_publish)
  int* d_seq = nullptr;                // device count of published states
  int seq = 0;                         // host count of lean graph launches
  // graph chunk
  hipGraphExec_t chunk_exec = nullptr;
  hipGraph_t chunk_graph = nullptr;
  int chunk_len = 0;
  // with the preconditioner (solve_lean): the head graph (start application, iterations
  // 1..L) and its continuation chunks; a group keeps its own
  LeanGraphs lean;
  // profiling
  bool prof = false;
  double spmv_ms = 0.0, asm_ms = 0.0;
  int64_t spmv_cnt = 0, asm_cnt = 0;
  hipEvent_t ev[2] = {nullptr, nullptr};
  // direct solve profiling: event pairs of up, top, down, residual; summed times, launches
  hipEvent_t dev[8] = {};
  double dir_ms[4] = {0.0, 0.0, 0.0, 0.0};
  int64_t dir_cnt = 0;
  std::vector<hipEvent_t> ev_pool;  // SpMV timing pairs inside one convergence chunk
  int prof_k = 0;
  // multi-rank: halo plan (nx_set_halo) and transport -- an RCCL communicator (one
  // process per GPU) or membership of an in-process group (nx_group_create)
  ncclComm_t comm = nullptr;
  nx_group* group = nullptr;
  hipStream_t own_stream = nullptr;  // the handle's stream while it is lent to a group
  int nranks = 1, rank = 0;
  bool have_plan = false;
  std::vector<int> peers, send_off, recv_off;
  std::vector<int> peer_src_off;  // group: offset of my segment in each peer's send_buf
  int* send_idx = nullptr;
  double* send_buf = nullptr;
  // beta^2 partials of all ranks (nranks), gathered point-to-point with the halo so the
  // iteration needs no separate all-reduce for it
  double* gath = nullptr;
  bool beta_p2p = true;
  bool rccl_graph_ok = true;  // capture of the RCCL iteration worked (or was not tried)
  bool sched_checked = false; // RCCL: the ranks' kernel schedules were compared (per pc)
  bool direct_all = false;    // RCCL: every rank can run the direct solve (check_schedules)
  bool last_graph = false;    // the last nx_solve replayed HIP graphs
  // solver (nx_set_solver): 0 = MINRES, 1 = direct tree solve where it is exact (one rank,
  // exact preconditioner on a forest: tree_exact from the host decomposition), else MINRES
  int solver = 0;
  bool tree_exact = false;
  int last_solver = 0;        // what the last nx_solve ran (0 MINRES, 1 direct)
  int pend_lhs = 0, pend_rhs = 0;  // deferred nx_assemble (flush_assembly)
  // direct solve, one rank: the residual check fused into the down sweep (PcArgs::fres);
  // the rows it cannot form (left, n_left) and ||b||^2 of the first pass (dir_bb)
  bool fres_ok = false;
  int top_ts0 = 0, top_nt = 0;  // the top part's slots (host copy of top_lvl_off's ends)
  int force_global = 0;  // nx_set_pc_kernels: the global-memory sweeps even where LDS fits
  int n_cu = 0;  // compute units of the device (topdown / coarsedown need one round of jobs)
  int* d_left = nullptr;
  int n_left = 0;
  double* dir_bb = nullptr;
  // the fused direct step (k_dir_step, one rank): per chain the post slots of its ends at
  // rows no job forms, every left row's post range, the posts, the hand-off counters and
  // the launches since they were zero (all in pc_bufs; reset with every upload)
  bool dstep_ok = false;   // the decomposition allows it (nx_set_preconditioner)
  bool dstep_multi = false;  // some job of the one-launch step needs several chain passes
  bool dq_stale = false;   // the last assembly was a one-launch step's: dq not formed (ensure_dq)
  bool dstep_off = false;  // a launch gave up waiting (workgroups not co-resident)
  int* d_chain_post = nullptr;
  int* d_left_off = nullptr;
  double* d_post = nullptr;
  unsigned* d_dsync = nullptr;
  unsigned dstep_epoch = 0;
  unsigned dstep_polls = kDirWaitPolls;  // the wait bound (nx_debug_set_wait_polls: tests)
  // k_dir_step's job headers, chain records (crec / ci: refreshed with the coefficients),
  // stash strides and dynamic LDS split (all in pc_bufs; nx_set_preconditioner)
  int* d_job_hdr = nullptr;
  double* d_crec = nullptr;
  int* d_ci = nullptr;
  int dstep_main = 0, dstep_top = 0;
  // several ranks (k_dir_xr / k_dir_xg, round 4): the fused step's tables hold (xr_ok); the
  // publisher's own left rows (xr_nleft: the left rows that are not cut); this
  // rank's mailbox (fine-grained; one block: mb1 | mb2 | flags), the peers' (device table,
  // IPC-mapped for RCCL ranks), the launch tag; host copies of the cut lists
  bool xr_ok = false;
  int xr_nleft = 0;
  void* xmb = nullptr;
  XPeer* d_xpeers = nullptr;
  std::vector<XPeer> xpeers_host;  // the same table on the host
  std::vector<void*> xr_opened;  // peers' mailboxes opened by IPC (closed on destroy)
  bool xr_linked = false;        // the peer table is set (group create / nx_xch_import)
  bool xr_off = false;           // the ranks agreed to leave it (xr_agree): the graph path
  bool xr_all = false;           // RCCL: every rank can run the exchange step (check_schedules)
  unsigned xtag = 0;
  unsigned xpoll[2] = {kDirWaitPolls, kDirWaitPolls};  // per exchange (nx_debug_xr_polls)
  unsigned xr_why = 0;        // the last exchange step's give-up reasons (kXrFail*), 0: none
  int xr_agreed = 0;          // agreements this handle took part in (nx_get_xr_status)
  double* d_agree = nullptr;  // RCCL: the agreement's all-reduce buffer
  // the host transport (tests: several ranks' processes on ONE GPU, nx_comm_init_host) --
  // the RCCL rank's host logic with its collectives through shared memory, eager only
  HostComm* hcomm = nullptr;
  std::vector<int> gk_off_host, gk_row_host;
  size_t dstep_lds = 0;  // dynamic LDS bytes per workgroup
  bool dstep_park = false;  // dstep_lds holds the superposition's park (DirStep::sup)
  bool dstep_rec = false;   // and the chain records' copy (sup & 4)
  bool last_sup = false;    // the last one-launch step ran the superposition instantiation
  unsigned* d_tsync = nullptr;  // k_dir_team_up's arrival counter (several ranks; pc_bufs)
  bool need_r = false;     // the last pass kept no residual: a refinement step forms it first
  int last_dir_path = 0;   // the last direct solve: 0 four launches, 1 k_dir_step
  std::vector<int> left_host;  // the rows of d_left
  // graphs with cycles (nx_set_cycles, one rank): the couplings the tree solve drops, as
  // row pairs (flux end, multiplier), and the Woodbury correction (k_cyc_*): Z (m = 2 n_cyc
  // columns of n_col), Cinv (m x m), U^T x before a refinement pass, w; rebuilt when the
  // matrix was assembled again (lhs_version)
  int n_cyc = 0;
  int* d_cyc_rows = nullptr;
  double* cyc_z = nullptr;
  double* cyc_cinv = nullptr;
  double* cyc_cap = nullptr;   // m x m, then m / 2 couplings
  double* cyc_gj = nullptr;    // cyc_invert's [A | I] (2 m^2) and its status word
  double* cyc_prev = nullptr;  // m
  double* cyc_w = nullptr;     // m
  bool cyc_raw = false;        // cyc_build's solves: the tree solve alone
  // several ranks (nx_set_cycles_team): per U column this rank's row or -1 (d_cyc_rows),
  // per pair the flux end row and the multiplier's column when the chain is here, else -1
  bool cyc_team = false;
  int* d_cyc_qloc = nullptr;
  int* d_cyc_lcol = nullptr;
  double* cyc_u = nullptr;  // m: U^T x summed over the ranks
  int64_t lhs_version = 0, cyc_version = -1;
  int64_t coef_version = 0, asm_coef_version = -1;  // nx_set_coefficients calls; at the last lhs
  // several ranks, direct (nx_set_cut): the multiplier rows of the K cut bifurcations are
  // completed inside the residual's all-reduce (no halo of x): per left row its cut index,
  // per cut index the owned row (or -1) and this rank's flux ends at it (row, +-1)
  int n_cut = -1;  // -1: not set
  std::vector<int> lm_cut;
  int* d_left_k = nullptr;
  int* d_cut_own = nullptr;
  int* d_gk_off = nullptr;
  int* d_gk_row = nullptr;
  double* d_gk_coef = nullptr;
  double* cutbuf = nullptr;  // [rr, bb, r_0 .. r_{K-1}] (all-reduced)
  // general element degrees (nx_create_fe): gather-assembly tables, one rank, no
  // preconditioner
  // nx_set_output_map: owned rows in the reference's function order (Solver.solve output)
  int* out_idx = nullptr;
  int64_t n_out = 0;
  // nx_snapshot_solution / nx_fetch_snapshot: device copies of x in the output order, the
  // event after each gather, the stream their device-to-host copies run on
  std::vector<double*> snap;
  std::vector<hipEvent_t> snap_ev;
  hipStream_t copy_stream = nullptr;
  bool fe = false;
  int* fe_kind = nullptr;
  double* fe_tval = nullptr;
  int* fe_aptr = nullptr;
  int* fe_aidx = nullptr;
  int* fe_aent = nullptr;
  int* fe_bptr = nullptr;
  int* fe_bidx = nullptr;
  int* fe_bent = nullptr;
  // (k, 0) solved through the condensed P1/DG0 system (nx_fe_set_direct): its handle (not
  // owned), the row maps, the cell constants C | K | Mii and a + b
  nx_network* fe_aux = nullptr;
  int fe_k = 0, fe_nl = 0;
  int fe_sk = 0;  // > 0: a (k, 0) layout whose terms fe_s_terms forms in closed form
  // (k, 0) edge templates (fe_build_tpl; k_fe_tasm / k_fe_tres): entries, shape offsets,
  // shape row starts, the edges' shapes and multiplier columns
  bool fe_tpl = false;
  int2* fe_tpl_buf = nullptr;   // packed entries (fe_tpl_pack)
  int2* fe_tpl_rbuf = nullptr;  // packed rhs terms
  int fe_tpl_off[9] = {};       // per shape (kFeShapes + 1)
  int fe_tpl_nsh = 0, fe_tpl_per = 0;
  int *fe_tpl_rs = nullptr, *fe_tpl_shape = nullptr, *fe_tpl_lam = nullptr;
  double* fe_cellh = nullptr;  // E*N cell lengths (k_fe_cellh at nx_create_fe)
  int *fe_slot = nullptr, *fe_vfe = nullptr, *fe_vaux = nullptr, *fe_ife = nullptr;
  int *fe_pfe = nullptr, *fe_paux = nullptr, *fe_lfe = nullptr, *fe_laux = nullptr;
  double* fe_cst = nullptr;
  double fe_ab = 0.0;
  hipEvent_t fe_ev[2] = {nullptr, nullptr};  // condensed rhs ready / auxiliary solve done
  // an auxiliary handle: its cell mass is a condensed one (nx_set_cell_mass), so its own CSR
  // is not the system the sweeps invert -- no residual check of its own
  bool cond_mass = false;
  // continuous pressure (k > m >= 1) on a forest: the node-condensed direct solve
  // (nx_fe_set_cp): reference blocks, per edge its border nodes, per border node its rows,
  // the node tree (levels, edges, parent, children), scratch (factors, Se | ge, node values)
  bool fe_cp = false;
  int cp_k = 0, cp_m = 0, cp_nI = 0, cp_nn = 0, cp_nlev = 0;
  double *cp_cst = nullptr, *cp_fac = nullptr, *cp_se = nullptr, *cp_xn = nullptr;
  double *cp_Pinv = nullptr, *cp_hv = nullptr;
  int *cp_tI = nullptr, *cp_eb = nullptr, *cp_nrow = nullptr, *cp_lev_off = nullptr;
  std::vector<int> cp_lev_host;  // the level offsets on the host (cp_nodes_launch)
  // runs of wide levels as subtree chunks (k_cp_nodes_rec, one workgroup per chunk): per run
  // its levels [L0, L1), its chunk count and its ranges' offset in cp_rng (2 (L1 - L0) ints
  // per chunk: each level's [start, end) in the records' level order)
  struct CpRun {
    int L0, L1, nch, off;
  };
  std::vector<CpRun> cp_runs;
  int* cp_rng = nullptr;
  std::vector<char> cp_lev_full;  // per level: every record holds its edges and children
  int *cp_order = nullptr, *cp_inc_off = nullptr, *cp_inc = nullptr, *cp_parent = nullptr;
  int *cp_child_off = nullptr, *cp_child = nullptr, *cp_nown = nullptr;
  // several ranks (nx_fe_cp_ranks): this rank's edges run the edge kernels (cp_Eown), every
  // rank's Se | ge (cp_Eg edges, by global edge: cp_gid) and node rhs (2 per node, after
  // them in cp_se) are summed over the ranks, the node forest is solved on every rank, and
  // each rank writes the node rows it owns (cp_nrowx: local rows, -1 elsewhere)
  int64_t cp_Eown = 0, cp_Eg = 0;
  int *cp_gid = nullptr, *cp_nrowx = nullptr;
  int* cp_rec = nullptr;  // the node records (CpTree::rec)
  double* cp_ctr = nullptr;  // the nodes' Schur terms for their parents (CpTree::ctr)
  std::vector<int> cp_gid_host, cp_nrowx_host;
};

struct nx_group {
  int P = 0;
  std::vector<nx_network*> hs;
  hipStream_t stream = nullptr;
  // k_dir_xg: the ranks' PcArgs / DirStep and workgroup offsets in device memory (pinned
  // staging: their contents change per launch -- the tags and sequence numbers)
  void* xg_dev = nullptr;
  void* xg_host = nullptr;
  hipGraphExec_t chunk_exec = nullptr;
  hipGraph_t chunk_graph = nullptr;
  int chunk_len = 0;
  LeanGraphs lean;
};

namespace {

int flush_assembly(nx_network* h);  // a deferred nx_assemble (defined with nx_assemble)

int grid_of(int64_t n, int per) { return (int)((n + per - 1) / per); }

template <class T>
int dalloc(T** p, int64_t count) {
  *p = nullptr;
  if (count <= 0) return NX_OK;
  HIPCALL(hipMalloc((void**)p, sizeof(T) * (size_t)count));
  return NX_OK;
}

template <class T>
int upload(T** p, const T* host, int64_t count, hipStream_t s) {
  CHECK(dalloc(p, count));
  if (count > 0) HIPCALL(hipMemcpyAsync(*p, host, sizeof(T) * count, hipMemcpyHostToDevice, s));
  return NX_OK;
}

Csr csr_of(const nx_network* h) { return Csr{h->rowptr, h->col, h->val, h->n_own}; }

// ---- transport. A Team is the set of handles one host thread drives in lock-step: one
// handle (single GPU, or one rank of an RCCL job) or all members of an in-process group
// (several ranks on one device, sharing one stream; exchanges are device copies).
struct Team {
  nx_network* const* hs;
  int P;
  nx_group* g;
};

// One rank of a job with one process per rank: an RCCL communicator, or the host transport.
bool proc_rank(const nx_network* h) { return h->comm != nullptr || h->hcomm != nullptr; }
bool team_multi(const Team& t) { return t.g != nullptr || proc_rank(t.hs[0]); }

// ---- the host transport (tests only) ----------------------------------------------------
// RCCL refuses two ranks on one device, so the RCCL ranks' host logic -- the exchange step's
// IPC mailboxes between processes, the agreement after a give-up (xr_agree), the graph
// path's collectives -- is tested on one GPU with the collectives through POSIX shared
// memory: a slot per rank, a sense-reversing barrier, sums in rank order (every rank gets
// the same bits, as k_group_sum). Every collective synchronises the handle's stream and
// copies through the host, so nothing is captured into graphs. Not a performance path.
constexpr size_t kHcHdr = 256;
constexpr size_t kHcSlot = 8u << 20;  // bytes per rank: the largest halo / all-reduce
constexpr double kHcTimeoutS = 300.0;

unsigned char* hc_slot(const HostComm* c, int r) { return c->base + kHcHdr + c->slot * (size_t)r; }

int hc_open(const std::string& name, int P, int rank, HostComm** out) {
  static_assert(std::atomic<uint32_t>::is_always_lock_free, "process-shared atomics");
  auto* c = new HostComm();
  c->P = P;
  c->rank = rank;
  c->slot = kHcSlot;
  c->bytes = kHcHdr + kHcSlot * (size_t)P;
  c->name = name;
  const int fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0) {
    delete c;
    return fail(NX_ERR_STATE, "host transport: shm_open(" + name + ") failed");
  }
  // (every rank sizes it the same; a fresh segment reads as zeros: the barrier's counters)
  void* p = ftruncate(fd, (off_t)c->bytes) == 0
                ? mmap(nullptr, c->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0)
                : MAP_FAILED;
  close(fd);
  if (p == MAP_FAILED) {
    delete c;
    return fail(NX_ERR_STATE, "host transport: mapping " + name + " failed");
  }
  c->base = static_cast<unsigned char*>(p);
  *out = c;
  return NX_OK;
}
void hc_close(HostComm* c) {
  if (!c) return;
  if (c->base) munmap(c->base, c->bytes);
  (void)shm_unlink(c->name.c_str());  // (the first rank to close removes the name)
  delete c;
}
int hc_barrier(HostComm* c) {
  auto* hd = reinterpret_cast<HcHdr*>(c->base);
  const uint32_t g = hd->gen.load(std::memory_order_acquire);
  if (hd->count.fetch_add(1u, std::memory_order_acq_rel) + 1u == (uint32_t)c->P) {
    hd->count.store(0u, std::memory_order_relaxed);
    hd->gen.store(g + 1u, std::memory_order_release);
    return NX_OK;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t k = 1; hd->gen.load(std::memory_order_acquire) == g; ++k) {
    if ((k & 255) == 0) {
      sched_yield();
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kHcTimeoutS)
        return fail(NX_ERR_STATE, "host transport: a rank never reached the barrier");
    }
  }
  return NX_OK;
}
// all-reduce of n values of T (device memory d) in rank order: op 0 sum, 1 max
template <class T>
int hc_allreduce(nx_network* h, T* d, int64_t n, int op) {
  HostComm* c = h->hcomm;
  if (sizeof(T) * (size_t)n > c->slot) return fail(NX_ERR_STATE, "host transport: all-reduce too large");
  HIPCALL(hipStreamSynchronize(h->stream));
  HIPCALL(hipMemcpy(hc_slot(c, c->rank), d, sizeof(T) * n, hipMemcpyDeviceToHost));
  CHECK(hc_barrier(c));
  std::vector<T> acc(reinterpret_cast<const T*>(hc_slot(c, 0)),
                     reinterpret_cast<const T*>(hc_slot(c, 0)) + n);
  for (int q = 1; q < c->P; ++q) {
    const T* s = reinterpret_cast<const T*>(hc_slot(c, q));
    for (int64_t i = 0; i < n; ++i) acc[i] = op == 0 ? acc[i] + s[i] : std::max(acc[i], s[i]);
  }
  CHECK(hc_barrier(c));  // (every rank has read the slots before they are written again)
  HIPCALL(hipMemcpy(d, acc.data(), sizeof(T) * n, hipMemcpyHostToDevice));
  return NX_OK;
}
// The halo of v (the pack kernels filled send_buf on the stream) and, beta, every rank's
// beta^2 partial (red[1]) into gath -- what team_halo's grouped send / recv moves. A slot
// holds [beta, n_peers, (peer, offset, count) per peer, send_buf]; every rank copies its
// segments out of its peers' slots.
int hc_halo(nx_network* h, double* v, bool beta) {
  HostComm* c = h->hcomm;
  const int np = (int)h->peers.size(), nsend = h->send_off.back();
  const size_t head = 2 + 3 * (size_t)np;
  if (sizeof(double) * (head + (size_t)nsend) > c->slot)
    return fail(NX_ERR_STATE, "host transport: halo too large");
  HIPCALL(hipStreamSynchronize(h->stream));
  double* s = reinterpret_cast<double*>(hc_slot(c, c->rank));
  s[0] = 0.0;
  if (beta) HIPCALL(hipMemcpy(s, h->red + 1, sizeof(double), hipMemcpyDeviceToHost));
  s[1] = np;
  for (int j = 0; j < np; ++j) {
    s[2 + 3 * j] = h->peers[j];
    s[3 + 3 * j] = h->send_off[j];
    s[4 + 3 * j] = h->send_off[j + 1] - h->send_off[j];
  }
  if (nsend > 0) HIPCALL(hipMemcpy(s + head, h->send_buf, sizeof(double) * nsend, hipMemcpyDeviceToHost));
  CHECK(hc_barrier(c));
  for (int j = 0; j < np; ++j) {
    const int cnt = h->recv_off[j + 1] - h->recv_off[j];
    if (cnt == 0) continue;
    const double* o = reinterpret_cast<const double*>(hc_slot(c, h->peers[j]));
    const int nq = (int)o[1];
    int e = 0;
    while (e < nq && (int)o[2 + 3 * e] != c->rank) ++e;
    if (e == nq || (int)o[4 + 3 * e] != cnt)
      return fail(NX_ERR_STATE, "host transport: the halo plans disagree");
    HIPCALL(hipMemcpy(v + h->n_own + h->recv_off[j], o + 2 + 3 * (size_t)nq + (size_t)o[3 + 3 * e],
                      sizeof(double) * cnt, hipMemcpyHostToDevice));
  }
  if (beta) {
    std::vector<double> g(c->P);
    HIPCALL(hipMemcpy(g.data(), h->gath, sizeof(double) * c->P, hipMemcpyDeviceToHost));
    for (int q = 0; q < c->P; ++q)
      if (q != c->rank) g[q] = reinterpret_cast<const double*>(hc_slot(c, q))[0];
    HIPCALL(hipMemcpy(h->gath, g.data(), sizeof(double) * c->P, hipMemcpyHostToDevice));
  }
  CHECK(hc_barrier(c));
  return NX_OK;
}

enum VecSel { VS_Z, VS_R2, VS_X };
double* vec_of(nx_network* h, VecSel s, int64_t k) {
  return s == VS_Z ? h->z : s == VS_X ? h->x : h->vb[k & 1];
}

// fill the ghost slots of the selected vector (n_col) from the owning ranks
int nB_of(const nx_network* h);

int team_halo(const Team& t, VecSel sel, int64_t k, bool beta = false, bool packed = false) {
  if (!team_multi(t)) return NX_OK;
  for (int r = 0; r < t.P && !packed; ++r) {  // packed: the down sweep's last workgroup did it
    nx_network* h = t.hs[r];
    const int nsend = h->send_off.back();
    if (beta)  // with the previous iteration's beta^2 partial sum
      hipLaunchKernelGGL(k_pack_beta, dim3(std::max(1, grid_of(nsend, kBlock))), dim3(kBlock), 0,
                         h->stream, vec_of(h, sel, k), h->send_idx, nsend, h->send_buf,
                         h->partB, nB_of(h), h->red + 1, h->gath + h->rank);
    else if (nsend > 0)
      hipLaunchKernelGGL(k_pack, dim3(grid_of(nsend, 256)), dim3(256), 0, h->stream,
                         vec_of(h, sel, k), h->send_idx, nsend, h->send_buf);
  }
  if (t.g) {
    for (int r = 0; r < t.P; ++r) {
      nx_network* h = t.hs[r];
      double* v = vec_of(h, sel, k);
      for (size_t j = 0; j < h->peers.size(); ++j) {
        const int cnt = h->recv_off[j + 1] - h->recv_off[j];
        if (cnt > 0)
          HIPCALL(hipMemcpyAsync(v + h->n_own + h->recv_off[j],
                                 t.hs[h->peers[j]]->send_buf + h->peer_src_off[j],
                                 sizeof(double) * cnt, hipMemcpyDeviceToDevice, h->stream));
      }
    }
    if (beta) {
      GroupPtrs src{}, dst{};
      for (int r = 0; r < t.P; ++r) {
        src.p[r] = t.hs[r]->red + 1;
        dst.p[r] = t.hs[r]->gath;
      }
      hipLaunchKernelGGL(k_group_gather, dim3(1), dim3(256), 0, t.hs[0]->stream, src, dst, t.P);
    }
    return NX_OK;
  }
  nx_network* h = t.hs[0];
  if (h->hcomm) return hc_halo(h, vec_of(h, sel, k), beta);
  if (h->peers.empty() && !beta) return NX_OK;
  double* v = vec_of(h, sel, k);
  NCCLCALL(ncclGroupStart());
  if (beta) {  // beta^2 partial to / from every other rank
    for (int q = 0; q < h->nranks; ++q) {
      if (q == h->rank) continue;
      NCCLCALL(ncclSend(h->red + 1, 1, ncclDouble, q, h->comm, h->stream));
      NCCLCALL(ncclRecv(h->gath + q, 1, ncclDouble, q, h->comm, h->stream));
    }
  }
  for (size_t p = 0; p < h->peers.size(); ++p) {
    const int sc = h->send_off[p + 1] - h->send_off[p];
    const int rc = h->recv_off[p + 1] - h->recv_off[p];
    if (sc > 0)
      NCCLCALL(ncclSend(h->send_buf + h->send_off[p], sc, ncclDouble, h->peers[p], h->comm,
                        h->stream));
    if (rc > 0)
      NCCLCALL(ncclRecv(v + h->n_own + h->recv_off[p], rc, ncclDouble, h->peers[p], h->comm,
                        h->stream));
  }
  NCCLCALL(ncclGroupEnd());
  return NX_OK;
}

// sum-all-reduce of n doubles: red + slot (slot 0..3), the coarse buffer (-1), the cut rows'
// buffer (-2), the cycle correction's U^T x (-3) or its U^T Z and couplings (-4), the
// continuous-pressure border blocks and node rhs (-5)
double* xbuf_of(nx_network* h, int slot) {
  return slot == -5 ? h->cp_se : slot == -4 ? h->cyc_cap : slot == -3 ? h->cyc_u
         : slot == -2 ? h->cutbuf : slot < 0 ? h->pa.cbuf : h->red + slot;
}

int team_allreduce(const Team& t, int slot, int n) {
  if (!team_multi(t) || n <= 0) return NX_OK;
  if (t.g) {
    GroupPtrs gp{};
    for (int r = 0; r < t.P; ++r) gp.p[r] = xbuf_of(t.hs[r], slot);
    hipLaunchKernelGGL(k_group_sum, dim3(std::min(grid_of(n, 256), 64)), dim3(256), 0,
                       t.hs[0]->stream, gp, t.P, n);
    return NX_OK;
  }
  nx_network* h = t.hs[0];
  if (h->hcomm) return hc_allreduce(h, xbuf_of(h, slot), n, 0);
  NCCLCALL(ncclAllReduce(xbuf_of(h, slot), xbuf_of(h, slot), n, ncclDouble, ncclSum, h->comm,
                         h->stream));
  return NX_OK;
}

// Columns of Gc (several ranks, once per solve after the start's coarse all-reduce): the
// coarse forest solve of e_k with this solve's D and G (k_pc_coarse's arithmetic), one
// workgroup per column. D and G are fixed for the solve, so z_c = Gc J_c afterwards.
constexpr int kGcThreads = 256;
__global__ __launch_bounds__(kGcThreads) void k_pc_gc(PcArgs pa) {
  __shared__ double sD[kCapCoarseLds], sJ[kCapCoarseLds], sZ[kCapCoarseLds];
  const int nC = pa.n_coarse, k = blockIdx.x;
  const double* __restrict__ G = pa.cbuf + 2 * nC;
  for (int i = threadIdx.x; i < nC; i += kGcThreads) {
    sD[i] = pa.cbuf[i];
    sJ[i] = i == k ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int lv = pa.n_clvl - 1; lv >= 0; --lv) {  // deepest level first
    for (int j = pa.c_lvl_off[lv] + threadIdx.x; j < pa.c_lvl_off[lv + 1]; j += kGcThreads) {
      double D = sD[j], J = sJ[j];
      for (int i = pa.c_child_off[j]; i < pa.c_child_off[j + 1]; ++i) {
        const int c = pa.c_child[i];
        const double g = G[c], Dc = sD[c];
        D -= g * g / Dc;
        J += g * sJ[c] / Dc;
      }
      sD[j] = D;
      sJ[j] = J;
    }
    __syncthreads();
  }
  for (int lv = 0; lv < pa.n_clvl; ++lv) {  // root level first
    for (int j = pa.c_lvl_off[lv] + threadIdx.x; j < pa.c_lvl_off[lv + 1]; j += kGcThreads) {
      const int p = pa.c_parent[j];
      sZ[j] = (sJ[j] + (p >= 0 ? G[j] * sZ[p] : 0.0)) / sD[j];
    }
    __syncthreads();
  }
  for (int j = threadIdx.x; j < nC; j += kGcThreads) pa.Gc[(int64_t)j * nC + k] = sZ[j];
}

// Preconditioner application on the stream: z = P^{-1} r' where r' = y - (alpha/beta) r2
// (mode 0, written back into y) or r' = y (mode 1, start). Partials of r'.z -> partB.
// half 0: chain condensation + junction elimination (up, top); half 1: back-substitution
// (top, down). With a coarse step the top kernel stops after the elimination, the coarse
// buffer is all-reduced between the halves and k_pc_coarse finishes the top part.
template <bool MULTI, int W, int CPL>
void launch_pc_wc(nx_network* h, double* y, const double* r2, MrState* st, MrState* other,
                  int mode, int half, double* zout, const hipEvent_t* evs) {
  // evs (profiling, LDS kernels): event pairs bound to the up / top / down dispatches
  const bool coarse = MULTI && h->pa.n_coarse > 0;
  double* const z = zout ? zout : h->z;
  hipEvent_t e[6] = {};
  if (evs)
    for (int i = 0; i < 6; ++i) e[i] = evs[i];
  if (half == 0) {
    if (h->pc_lds) {
      if (h->pc_jobs > 0)
        hipExtLaunchKernelGGL((k_pc_up_lds<MULTI, W, CPL>), dim3(h->pc_jobs), dim3(kPcThreads), 0,
                              h->stream, e[0], e[1], 0, h->pa, y, r2, st, other, h->partA, h->nA,
                              h->red, mode);
      if (MULTI && h->pa.mdense && mode == 0) {  // dense top: the coarse partials only
        if (!h->pa.fused)  // else the up sweep's last workgroup computes them
          hipLaunchKernelGGL(k_pc_cpart, dim3(1), dim3(kTopThreads), 0, h->stream, h->pa, st, mode);
      } else if (!(!MULTI && h->pa.dense && mode == 0) &&  // dense top: k_pc_down_lds does it
                 !(!MULTI && h->pa.topdown && mode == kModeDirect))  // so does topdown
        hipExtLaunchKernelGGL((k_pc_top_lds<MULTI>), dim3(1), dim3(kTopThreads), 0, h->stream, e[2],
                              e[3], 0, h->pa, y, r2, z, st, h->partA, h->nA, h->red, h->partB, mode);
    } else {
      if (h->pc_jobs > 0)
        hipLaunchKernelGGL((k_pc_up<MULTI, W, CPL>), dim3(h->pc_jobs), dim3(kBlock), 0, h->stream,
                           h->pa, y, r2, st, other, h->partA, h->nA, h->red, mode);
      hipLaunchKernelGGL((k_pc_top<MULTI>), dim3(1), dim3(kTopThreads), 0, h->stream, h->pa, y,
                         r2, z, st, h->partA, h->nA, h->red, h->partB, mode);
    }
    return;
  }
  // fused (dense top, LDS kernels): every down workgroup solves the coarse forest itself
  const bool cfused = MULTI && h->pc_lds && h->pa.fused && h->pa.mdense && mode == 0;
  if (coarse && !cfused && !(mode == kModeDirect && h->pa.coarsedown))
    hipLaunchKernelGGL(k_pc_coarse, dim3(1), dim3(kTopThreads), 0, h->stream, h->pa, y, r2, z,
                       st, h->partB, mode);
  if (h->pc_jobs > 0) {
    if (h->pc_lds && mode == kModeDirect && (MULTI ? h->pa.coarsedown : h->pa.topdown))
      hipExtLaunchKernelGGL((k_pc_down_lds<MULTI, W, CPL, true>), dim3(h->pc_jobs), dim3(kPcThreads),
                            0, h->stream, e[4], e[5], 0, h->pa, y, r2, z, st, h->partB, mode);
    else if (h->pc_lds && mode == kModeDirect)  // (the top part / coarse forest solved before)
      hipExtLaunchKernelGGL((k_pc_down_lds<MULTI, W, CPL, true, false>), dim3(h->pc_jobs),
                            dim3(kPcThreads), 0, h->stream, e[4], e[5], 0, h->pa, y, r2, z, st,
                            h->partB, mode);
    else if (h->pc_lds)
      hipExtLaunchKernelGGL((k_pc_down_lds<MULTI, W, CPL, false>), dim3(h->pc_jobs), dim3(kPcThreads),
                            0, h->stream, e[4], e[5], 0, h->pa, y, r2, z, st, h->partB, mode);
    else
      hipLaunchKernelGGL((k_pc_down<MULTI, W, CPL>), dim3(h->pc_jobs), dim3(kBlock), 0, h->stream,
                         h->pa, y, z, st, h->partB, mode);
  }
  // the iterations' dense coarse step: Gc is read only by the fused dense down sweep
  if (MULTI && coarse && mode == 1 && h->pa.Gc != nullptr && h->pc_lds && h->pa.fused &&
      h->pa.mdense)
    hipLaunchKernelGGL(k_pc_gc, dim3(h->pa.n_coarse), dim3(kGcThreads), 0, h->stream, h->pa);
}

template <bool MULTI>
void launch_pc(nx_network* h, double* y, const double* r2, MrState* st, MrState* other, int mode,
               int half, double* zout = nullptr, const hipEvent_t* evs = nullptr) {
  switch (h->pc_variant) {
    case 0: launch_pc_wc<MULTI, 16, 1>(h, y, r2, st, other, mode, half, zout, evs); break;
    case 1: launch_pc_wc<MULTI, 16, 2>(h, y, r2, st, other, mode, half, zout, evs); break;
    case 2: launch_pc_wc<MULTI, 16, 4>(h, y, r2, st, other, mode, half, zout, evs); break;
    case 3: launch_pc_wc<MULTI, 64, 2>(h, y, r2, st, other, mode, half, zout, evs); break;
    case 5: launch_pc_wc<MULTI, 8, 2>(h, y, r2, st, other, mode, half, zout, evs); break;
    case 6: launch_pc_wc<MULTI, 4, 4>(h, y, r2, st, other, mode, half, zout, evs); break;
    case 7: launch_pc_wc<MULTI, 8, 4>(h, y, r2, st, other, mode, half, zout, evs); break;
    case 8: launch_pc_wc<MULTI, 64, 8>(h, y, r2, st, other, mode, half, zout, evs); break;
    case 9: launch_pc_wc<MULTI, 64, 16>(h, y, r2, st, other, mode, half, zout, evs); break;
    default: launch_pc_wc<MULTI, 64, 4>(h, y, r2, st, other, mode, half, zout, evs); break;
  }
}

int nB_of(const nx_network* h) { return h->pc ? h->pc_jobs + 1 : h->nB; }

bool team_lin(const Team& t) {
  const nx_network* h = t.hs[0];
  return team_multi(t) && h->pc && h->pa.n_coarse > 0 && h->pa.lin;
}


// Whole preconditioner application for every rank of the team, with the coarse exchange.
// from_rhs: the start condenses the rhs itself and iteration 1 reads r_1 = b from it (the
// one-graph solve; the rhs is read-only for both)
int team_pc(const Team& t, int64_t k, int mode, bool from_rhs = false) {
  const bool multi = team_multi(t);
  for (int half = 0; half < 2; ++half) {
    for (int r = 0; r < t.P; ++r) {
      nx_network* h = t.hs[r];
      double* y = mode ? (from_rhs ? h->rhs : h->vb[0]) : h->vb[(k - 1) & 1];
      const double* r2 = mode ? h->vb[1] : (from_rhs && k == 1) ? h->rhs : h->vb[k & 1];
      MrState* st = mode ? h->st : h->st + (k & 1);
      MrState* other = mode ? h->st + 1 : h->st + ((k + 1) & 1);
      if (multi) launch_pc<true>(h, y, r2, st, other, mode, half);
      else launch_pc<false>(h, y, r2, st, other, mode, half);
    }
    if (half == 0 && multi && t.hs[0]->pa.n_coarse > 0)
      CHECK(team_allreduce(t, -1, 3 * t.hs[0]->pa.n_coarse + (team_lin(t) ? 1 : 0)));
  }
  return NX_OK;
}

int team_reduce_slot(const Team& t, bool from_a, int slot, bool allreduce = true) {
  // linear form: alpha's partial goes into the coarse buffer and is reduced with it; the
  // up kernel's workgroup 0 sums it (no launch here) when the rank has LDS jobs
  const bool to_coarse = from_a && slot == 0 && team_lin(t);
  for (int r = 0; r < t.P; ++r) {
    nx_network* h = t.hs[r];
    if (to_coarse && h->pc_lds && h->pc_jobs > 0) continue;
    hipLaunchKernelGGL(k_reduce_slot, dim3(1), dim3(kBlock), 0, h->stream,
                       from_a ? h->partA : h->partB, from_a ? h->nA : nB_of(h),
                       to_coarse ? h->pa.cbuf + 3 * h->pa.n_coarse : h->red, to_coarse ? 0 : slot);
  }
  return (to_coarse || !allreduce) ? NX_OK : team_allreduce(t, slot, 1);
}

// Lean graphs: k_mr_a of iteration 1 initialises the state; the graph's last k_mr_a
// publishes its state (MrInit).
struct LeanOpt {
  bool init, mark;
  double rtol;
  int maxit;
};

// First part of MINRES iteration k (1-based) of every rank on the stream: the halo (with
// several ranks also the previous beta^2 partial), then k_mr_a.
int launch_part_a(const Team& t, int64_t k, const LeanOpt* lo = nullptr) {
  const bool multi = team_multi(t);
  const bool pc = t.hs[0]->pc;
  // beta^2 of the previous iteration travels with the halo (point-to-point gather)
  const bool p2p_beta = multi && t.hs[0]->beta_p2p;
  const bool packed = lo != nullptr && k >= 2 && pc && t.hs[0]->pa.fuse_pack;
  if (multi) CHECK(team_halo(t, pc ? VS_Z : VS_R2, k, p2p_beta, packed));
  for (int r = 0; r < t.P; ++r) {
    nx_network* h = t.hs[r];
    double* r1 = h->vb[(k - 1) & 1];
    double* r2 = h->vb[k & 1];
    // pending update of iteration k-1: w1 = w_{k-3} (overwritten by w_{k-1}), w2 = w_{k-2}
    double* w1 = h->wb[k & 1];
    double* w2 = h->wb[(k - 1) & 1];
    MrState* sin = h->st + ((k + 1) & 1);
    MrState* sout = h->st + (k & 1);
    // one-graph solve: k_mr_a(2) reads r_1 = b from the rhs
    MrVecs mv{r1,   (lo && pc && k == 2) ? h->rhs : r1, r2, w1, w2, h->x, h->z, h->vv,
              pc ? h->vs : nullptr, h->n_own, h->hist};
    const int nB = nB_of(h);
    // profiling (single handle): events bound to the kernel's own dispatch packet
    // (hipExtLaunchKernel), so the interval is the kernel's execution like rocprofv3's
    const bool prof = h->prof && t.g == nullptr;
    hipEvent_t e0 = prof ? h->ev_pool[2 * h->prof_k] : nullptr;
    hipEvent_t e1 = prof ? h->ev_pool[2 * h->prof_k + 1] : nullptr;
    const double* bpart = p2p_beta ? h->gath : h->partB;
    const int nbp = p2p_beta ? h->nranks : nB;
    MrInit ini{0, 0, 0, 0.0, nullptr, 0, nullptr, nullptr};
    if (lo)
      ini = MrInit{lo->init ? 1 : 0, nbp, lo->maxit, lo->rtol, bpart, lo->mark ? 1 : 0,
                   h->d_seq, h->d_last};
#define NX_LAUNCH_A(M, P)                                                                        \
  hipExtLaunchKernelGGL((k_mr_a<M, P>), dim3(h->nA), dim3(kBlock), 0, h->stream, e0, e1, 0,     \
                        csr_of(h), mv, sin, sout, bpart, nbp, h->red, h->partA, h->chunksA, ini)
    if (multi && !p2p_beta) {
      if (pc) NX_LAUNCH_A(true, true); else NX_LAUNCH_A(true, false);
    } else {
      if (pc) NX_LAUNCH_A(false, true); else NX_LAUNCH_A(false, false);
    }
#undef NX_LAUNCH_A
    if (prof) h->prof_k += 1;
  }
  if (multi) CHECK(team_reduce_slot(t, true, 0));
  HIPCALL(hipGetLastError());
  return NX_OK;
}

// Second part of iteration k: the preconditioner (or the Lanczos step without it) and,
// with several ranks and beta^2 by all-reduce, that reduction.
int launch_part_pc(const Team& t, int64_t k, bool from_rhs = false) {
  const bool multi = team_multi(t);
  const bool pc = t.hs[0]->pc;
  const bool p2p_beta = multi && t.hs[0]->beta_p2p;
  if (pc) {
    CHECK(team_pc(t, k, 0, from_rhs));
  } else {
    for (int r = 0; r < t.P; ++r) {
      nx_network* h = t.hs[r];
      double* r1 = h->vb[(k - 1) & 1];
      double* r2 = h->vb[k & 1];
      MrState* sin = h->st + ((k + 1) & 1);
      MrState* sout = h->st + (k & 1);
      if (multi)
        hipLaunchKernelGGL(k_mr_b<true>, dim3(h->nB), dim3(kBlock), 0, h->stream, h->n_own, r1, r2,
                           sout, sin, h->partA, h->nA, h->red, h->partB);
      else
        hipLaunchKernelGGL(k_mr_b<false>, dim3(h->nB), dim3(kBlock), 0, h->stream, h->n_own, r1,
                           r2, sout, sin, h->partA, h->nA, h->red, h->partB);
    }
  }
  if (multi && !p2p_beta) CHECK(team_reduce_slot(t, false, 1));  // p2p: k_pack_beta sums
  HIPCALL(hipGetLastError());
  return NX_OK;
}

// One MINRES iteration of every rank on the stream; `k` = 1-based iteration index.
int launch_iteration(const Team& t, int64_t k) {
  CHECK(launch_part_a(t, k));
  return launch_part_pc(t, k);
}

struct GraphSlot {
  hipGraphExec_t* exec;
  hipGraph_t* graph;
  int* len;
  LeanGraphs* lean;  // the head / continuation graphs of the same handle or group go too
};

GraphSlot graph_slot(const Team& t) {
  if (t.g) return GraphSlot{&t.g->chunk_exec, &t.g->chunk_graph, &t.g->chunk_len, &t.g->lean};
  nx_network* h = t.hs[0];
  return GraphSlot{&h->chunk_exec, &h->chunk_graph, &h->chunk_len, &h->lean};
}

int drop_one(hipGraphExec_t* exec, hipGraph_t* graph, int* len) {
  if (*exec) HIPCALL(hipGraphExecDestroy(*exec));
  if (*graph) HIPCALL(hipGraphDestroy(*graph));
  *exec = nullptr;
  *graph = nullptr;
  *len = 0;
  return NX_OK;
}

int drop_graph(GraphSlot gs) {
  CHECK(drop_one(gs.exec, gs.graph, gs.len));
  if (gs.lean) {
    CHECK(drop_one(&gs.lean->head_exec, &gs.lean->head_graph, &gs.lean->head_len));
    CHECK(drop_one(&gs.lean->lchunk_exec, &gs.lean->lchunk_graph, &gs.lean->lchunk_len));
    CHECK(drop_one(&gs.lean->direct_exec, &gs.lean->direct_graph, &gs.lean->direct_len));
    CHECK(drop_one(&gs.lean->direct_asm_exec, &gs.lean->direct_asm_graph,
                   &gs.lean->direct_asm_len));
  }
  return NX_OK;
}

// Captured launches bake in a handle's arguments: after a change, drop the handle's graphs
// and those of the group it belongs to.
int drop_handle_graphs(nx_network* h) {
  nx_network* hs[1] = {h};
  CHECK(drop_graph(graph_slot(Team{hs, 1, nullptr})));
  if (h->group) {
    nx_group* g = h->group;
    CHECK(drop_graph(GraphSlot{&g->chunk_exec, &g->chunk_graph, &g->chunk_len, &g->lean}));
  }
  return NX_OK;
}

int build_chunk_graph(const Team& t, int len) {
  GraphSlot gs = graph_slot(t);
  if (*gs.exec && *gs.len == len) return NX_OK;
  CHECK(drop_graph(gs));
  hipStream_t s = t.hs[0]->stream;
  HIPCALL(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  int rc = NX_OK;
  for (int j = 0; j < len && rc == NX_OK; ++j) rc = launch_iteration(t, j + 1);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(s, &g);
  if (rc != NX_OK) return rc;
  if (e != hipSuccess) return fail(NX_ERR_HIP, std::string("capture: ") + hipGetErrorString(e));
  *gs.graph = g;
  HIPCALL(hipGraphInstantiate(gs.exec, g, nullptr, nullptr, 0));
  *gs.len = len;
  return NX_OK;
}

int set_device(nx_network* h) {
  HIPCALL(hipSetDevice(h->device));
  return NX_OK;
}

// Pivots of the P1 mass matrix of one edge, M_e = (R h / 6) T, T = tridiag(1, 4, 1) of size
// N+1 with 2 at both ends (assembly.py:253 on equal cells): T = L U with unit lower
// multipliers l_k = 1 / u_{k-1} (l_0 = 0) and pivots u_0 = 2, u_k = d_k - l_k.
// Returns [l_0..l_N | 1/u_0..1/u_N].
// ratio = a / b of the cell mass (P1: 2): T = M / (b R h) = tridiag(1, 2 ratio, 1) with ratio
// at both ends
std::vector<double> mass_lu(int N, double ratio = 2.0) {
  const int n = N + 1;
  std::vector<double> lu(2 * (size_t)n, 0.0);
  double u = ratio;
  lu[n] = 1.0 / u;
  for (int k = 1; k < n; ++k) {
    const double l = 1.0 / u;
    u = (k == N ? ratio : 2.0 * ratio) - l;
    lu[k] = l;
    lu[n + k] = 1.0 / u;
  }
  return lu;
}

}  // namespace

// ======================================================================================
// C ABI
// ======================================================================================

NX_API int nx_version(void) { return kVersion; }

NX_API const char* nx_last_error(void) { return g_err.c_str(); }

NX_API int nx_device_count(int32_t* count) {
  int n = 0;
  HIPCALL(hipGetDeviceCount(&n));
  *count = n;
  return NX_OK;
}

NX_API int nx_create(int32_t device, int32_t N, int64_t n_edges, const double* edge_x,
                     const int32_t* edge_lm, int64_t n_lm, const int32_t* lm_rowptr,
                     const int32_t* lm_col, const double* lm_val, int64_t n_ghost,
                     nx_network_t** out) {
  if (out == nullptr) return fail(NX_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (N < 1) return fail(NX_ERR_ARG, "N must be >= 1");
  if (n_edges < 0 || n_lm < 0 || n_ghost < 0) return fail(NX_ERR_ARG, "negative size");
  if (n_edges > 0 && (edge_x == nullptr || edge_lm == nullptr))
    return fail(NX_ERR_ARG, "edge arrays are NULL");
  if (n_lm > 0 && (lm_rowptr == nullptr || lm_col == nullptr || lm_val == nullptr))
    return fail(NX_ERR_ARG, "multiplier arrays are NULL");
  const int64_t per = 2 * (int64_t)N + 1;
  const int64_t n_edge_dofs = n_edges * per;
  const int64_t n_own = n_edge_dofs + n_lm;
  const int64_t n_col = n_own + n_ghost;
  // segment offsets (host prefix sum), 32-bit CSR indices
  std::vector<int> seg((size_t)n_edges + 1);
  int64_t acc = 0;
  for (int64_t e = 0; e < n_edges; ++e) {
    seg[e] = (int)acc;
    const int a = edge_lm[2 * e], b = edge_lm[2 * e + 1];
    if (a >= n_col || b >= n_col || (a >= 0 && a < n_edge_dofs) || (b >= 0 && b < n_edge_dofs))
      return fail(NX_ERR_ARG, "edge_lm column out of range (must be a multiplier or ghost column)");
    acc += 7 * (int64_t)N + 1 + (a >= 0) + (b >= 0);
  }
  seg[n_edges] = (int)acc;
  const int64_t nnz_lm = n_lm > 0 ? lm_rowptr[n_lm] : 0;
  if (n_lm > 0 && lm_rowptr[0] != 0) return fail(NX_ERR_ARG, "lm_rowptr[0] must be 0");
  for (int64_t i = 0; i < nnz_lm; ++i)
    if (lm_col[i] < 0 || lm_col[i] >= n_col) return fail(NX_ERR_ARG, "lm_col out of range");
  if (acc + nnz_lm >= (int64_t)INT32_MAX || n_col >= (int64_t)INT32_MAX)
    return fail(NX_ERR_ARG, "problem too large for 32-bit CSR indices on one rank");

  int ndev = 0;
  HIPCALL(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev)
    return fail(NX_ERR_ARG, "device " + std::to_string(device) + " not visible (" +
                                std::to_string(ndev) + " devices)");
  HIPCALL(hipSetDevice(device));

  auto* h = new nx_network();
  h->device = device;
  h->N = N;
  h->E = n_edges;
  h->B = n_lm;
  h->n_edge_dofs = n_edge_dofs;
  h->n_own = n_own;
  h->n_ghost = n_ghost;
  h->n_col = n_col;
  h->nnz_edges = acc;
  h->nnz_lm = nnz_lm;
  h->nnz = acc + nnz_lm;
  h->nblk = std::max(1, grid_of(n_own, kRowsPerBlock));  // >= 1: every rank joins the reductions
  auto bail = [&](int rc) {
    nx_destroy(h);
    return rc;
  };
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return bail(fail(NX_ERR_HIP, "hipStreamCreate failed"));
  int rc = NX_OK;
  if ((rc = upload(&h->edge_x, edge_x, 6 * n_edges, h->stream))) return bail(rc);
  if ((rc = upload(&h->edge_lm, edge_lm, 2 * n_edges, h->stream))) return bail(rc);
  if ((rc = upload(&h->edge_seg, seg.data(), n_edges + 1, h->stream))) return bail(rc);
  if ((rc = upload(&h->lm_val, lm_val, nnz_lm, h->stream))) return bail(rc);
  if ((rc = dalloc(&h->edge_R, n_edges))) return bail(rc);
  if ((rc = dalloc(&h->edge_bc, 2 * n_edges))) return bail(rc);
  if ((rc = dalloc(&h->dq, n_edges * (int64_t)(N + 1)))) return bail(rc);
  if ((rc = dalloc(&h->rowptr, n_own + 1))) return bail(rc);
  if ((rc = dalloc(&h->col, h->nnz))) return bail(rc);
  if ((rc = dalloc(&h->val, h->nnz))) return bail(rc);
  // rhs has ghost slots (zero): the one-graph solve reads b as r_1 straight from it, and the
  // junction slots of ghost junctions index past the owned rows
  if ((rc = dalloc(&h->rhs, n_col))) return bail(rc);
  if (n_col > n_own && hipMemsetAsync(h->rhs + n_own, 0, sizeof(double) * (n_col - n_own),
                                      h->stream) != hipSuccess)
    return bail(fail(NX_ERR_HIP, "memset failed"));
  for (int i = 0; i < 2; ++i) {
    if ((rc = dalloc(&h->vb[i], n_col))) return bail(rc);
    if ((rc = dalloc(&h->wb[i], n_own))) return bail(rc);
    // the ghost slots of r are read (junction slots of ghost junctions) and must stay zero
    if (n_col > 0 && hipMemsetAsync(h->vb[i], 0, sizeof(double) * n_col, h->stream) != hipSuccess)
      return bail(fail(NX_ERR_HIP, "memset failed"));
  }
  if ((rc = dalloc(&h->x, n_col))) return bail(rc);
  if ((rc = dalloc(&h->tmp, n_col))) return bail(rc);
  h->nA = std::max(1, grid_of(n_own, kRowsPerBlock * h->chunksA));
  if ((rc = dalloc(&h->partials, 2 * (int64_t)h->nblk))) return bail(rc);
  if ((rc = dalloc(&h->partA, h->nA))) return bail(rc);
  if ((rc = dalloc(&h->partB, h->nB))) return bail(rc);
  if ((rc = dalloc(&h->red, 4))) return bail(rc);
  if (hipMalloc((void**)&h->st, 2 * sizeof(MrState)) != hipSuccess)
    return bail(fail(NX_ERR_HIP, "hipMalloc state failed"));
  if (hipHostMalloc((void**)&h->h_last, sizeof(MrState),
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&h->d_last, h->h_last, 0) != hipSuccess)
    return bail(fail(NX_ERR_HIP, "mapped host state allocation failed"));
  std::memset(h->h_last, 0, sizeof(MrState));
  if ((rc = dalloc(&h->d_seq, 1))) return bail(rc);
  if (hipMemsetAsync(h->d_seq, 0, sizeof(int), h->stream) != hipSuccess)
    return bail(fail(NX_ERR_HIP, "memset failed"));
  if (hipHostMalloc((void**)&h->h_st, 2 * sizeof(MrState), hipHostMallocDefault) != hipSuccess)
    return bail(fail(NX_ERR_HIP, "hipHostMalloc failed"));
  for (auto& e : h->ev)
    if (hipEventCreate(&e) != hipSuccess) return bail(fail(NX_ERR_HIP, "hipEventCreate failed"));
  if (hipMemsetAsync(h->st, 0, 2 * sizeof(MrState), h->stream) != hipSuccess)
    return bail(fail(NX_ERR_HIP, "memset state failed"));

  if (hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    h->n_cu = 0;
  // pattern: edge segments on the device; multiplier rows from the host lists
  if (n_edges > 0) {
    EdgeArgs ea{h->edge_x, h->edge_lm, h->edge_seg, n_edges, N};
    hipLaunchKernelGGL(k_pattern, dim3(grid_of(n_edges, kBlock / 64)), dim3(kBlock), 0, h->stream,
                       ea, h->rowptr, h->col);
  }
  std::vector<int> rp_lm((size_t)n_lm + 1);
  for (int64_t b = 0; b <= n_lm; ++b) rp_lm[b] = (int)(acc + (n_lm > 0 ? lm_rowptr[b] : 0));
  if (hipMemcpyAsync(h->rowptr + n_edge_dofs, rp_lm.data(), sizeof(int) * (n_lm + 1),
                     hipMemcpyHostToDevice, h->stream) != hipSuccess)
    return bail(fail(NX_ERR_HIP, "rowptr upload failed"));
  if (nnz_lm > 0 && hipMemcpyAsync(h->col + acc, lm_col, sizeof(int) * nnz_lm,
                                   hipMemcpyHostToDevice, h->stream) != hipSuccess)
    return bail(fail(NX_ERR_HIP, "lm col upload failed"));
  if (hipGetLastError() != hipSuccess) return bail(fail(NX_ERR_HIP, "pattern kernel launch failed"));
  if (hipStreamSynchronize(h->stream) != hipSuccess)
    return bail(fail(NX_ERR_HIP, "pattern build failed"));
  *out = h;
  return NX_OK;
}

// ---- general element degrees (HydraulicNetworkAssembler(flux_degree=k, pressure_degree=m),
// assembly.py:121-146). The host lists every nonzero's and every rhs row's terms in a
// fixed order (layout_fe.py); k_assemble_fe evaluates them, one thread per nonzero / row.
// Deterministic: same terms, same order on every call, no atomics.
namespace {

enum FeKind : int { kFeConst = 0, kFeMass = 1, kFeSource = 2, kFeBc = 3 };

struct FeArgs {
  const double* edge_x;  // E*6
  const double* edge_R;  // E
  const double* edge_bc; // E*2
  double f;
  const double* edge_f;  // E per-edge source, or nullptr: f everywhere
  int N;
  const int* kind;       // term table
  const double* tval;
  const int* a_ptr;      // nnz + 1
  const int* a_idx;
  const int* a_ent;
  const int* b_ptr;      // n_rows + 1
  const int* b_idx;
  const int* b_ent;
  int64_t nnz, n_rows;
  double* val;
  double* rhs;
  int lhs, do_rhs;
  int64_t n_edges;  // (k_fe_tasm)
  const double* cellh;  // E*N cell lengths (fe_cell_h, once per handle), or null: formed here
};

// length of cell c of edge e, vertices generated like the reference mesh (mesh.py:275-291)
__device__ __forceinline__ double fe_cell_h(const double* __restrict__ edge_x, int64_t cell, int N) {
#pragma clang fp contract(off)
  const int64_t e = cell / N;
  const int c = (int)(cell - e * N);
  const double invN = 1.0 / (double)N;
  double x0[3], x1[3], pa[3], pb[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    x0[d] = edge_x[6 * e + d];
    x1[d] = edge_x[6 * e + 3 + d];
  }
  vertex(x0, x1, c, N, invN, pa);
  vertex(x0, x1, c + 1, N, invN, pb);
  const double d0 = pb[0] - pa[0], d1 = pb[1] - pa[1], d2 = pb[2] - pa[2];
  return sqrt(d0 * d0 + d1 * d1 + d2 * d2);
}

__device__ __forceinline__ double fe_term(const FeArgs& a, int idx, int ent) {
#pragma clang fp contract(off)
  const double v = a.tval[ent];
  switch (a.kind[ent]) {
    case kFeMass:
      return (a.edge_R[idx / a.N] * (a.cellh ? a.cellh[idx] : fe_cell_h(a.edge_x, idx, a.N))) * v;
    case kFeSource:
      return ((a.edge_f ? a.edge_f[idx / a.N] : a.f) *
              (a.cellh ? a.cellh[idx] : fe_cell_h(a.edge_x, idx, a.N))) * v;
    case kFeBc: return a.edge_bc[idx] * v;
    default: return v;
  }
}

// every cell's length once per handle (the geometry is fixed at nx_create_fe): the gathered
// mass and source terms read it instead of forming both vertices per term (the same bits)
__global__ __launch_bounds__(kBlock) void k_fe_cellh(const double* __restrict__ edge_x, int N,
                                                     int64_t n_cells, double* __restrict__ out) {
  const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (c < n_cells) out[c] = fe_cell_h(edge_x, c, N);
}

__global__ __launch_bounds__(kBlock) void k_assemble_fe(FeArgs a) {
#pragma clang fp contract(off)
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (a.lhs && t < a.nnz) {
    double s = 0.0;
    for (int c = a.a_ptr[t]; c < a.a_ptr[t + 1]; ++c) s += fe_term(a, a.a_idx[c], a.a_ent[c]);
    a.val[t] = s;
  }
  if (a.do_rhs && t < a.n_rows) {
    double s = 0.0;
    for (int c = a.b_ptr[t]; c < a.b_ptr[t + 1]; ++c) s += fe_term(a, a.b_idx[c], a.b_ent[c]);
    a.rhs[t] = s;
  }
}

// (k, 0) layouts (layout_fe.py with m = 0): the terms of entry (row, col) in closed form --
// the same (index, table entry) list, in the same order, as the host's gather tables, which
// nx_create_fe checks entry by entry before it builds the edge templates (fe_build_tpl).
// Per edge e: kN + 1 flux rows then N cell pressure rows (per = kN + 1 + N); the multiplier
// rows after all edges. Table: (k+1)^2 mass, k+1 divergence, +1, -1, source, bc.
struct FeTerm {
  int idx, ent;
};
// an edge row's terms: pos its row and lc its column within the edge (0 .. per-1), or lc = -1
// for a multiplier column, -2 for another edge's; c0 = the edge's first cell
__host__ __device__ __forceinline__ int fe_s_terms_loc(int pos, int lc, int k, int N, int c0,
                                                       FeTerm* out) {
  const int nq = k + 1, nf = k * N + 1;
  const int ent_b = nq * nq, ent_plus = nq * nq + nq, ent_minus = ent_plus + 1;
  if (lc == -1) {  // a flux end's multiplier column
    if (pos == nf - 1) out[0] = FeTerm{0, ent_plus};
    else if (pos == 0) out[0] = FeTerm{0, ent_minus};
    else return 0;
    return 1;
  }
  if (lc < 0) return 0;
  if (pos >= nf) {  // a pressure row: divergence of its cell's flux nodes
    const int c = pos - nf, i = lc - c * k;
    if (lc >= nf || i < 0 || i > k) return 0;
    out[0] = FeTerm{c0 + c, ent_b + i};
    return 1;
  }
  if (lc >= nf) {  // a flux row's gradient entry
    const int c = lc - nf, i = pos - c * k;
    if (i < 0 || i > k) return 0;
    out[0] = FeTerm{c0 + c, ent_b + i};
    return 1;
  }
  // flux-flux mass: the cells holding both nodes, by reference entry then cell (generation order)
  int n = 0;
  FeTerm t[2];
  int blk[2];
  const int pk = pos / k;
  for (int side = 0; side < 2; ++side) {
    const int c = side == 0 ? pk : pk - 1;  // the cell on the right / left of the node
    if (c < 0 || c >= N || (side == 1 && pos - pk * k != 0)) continue;
    const int i = pos - c * k, j = lc - c * k;
    if (j < 0 || j > k) continue;
    t[n] = FeTerm{c0 + c, i * nq + j};
    blk[n] = i * nq + j;
    ++n;
  }
  if (n == 2 && (blk[1] < blk[0] || (blk[1] == blk[0] && t[1].idx < t[0].idx))) {
    out[0] = t[1];
    out[1] = t[0];
  } else {
    for (int q = 0; q < n; ++q) out[q] = t[q];
  }
  return n;
}
__host__ __device__ __forceinline__ int fe_s_terms(int64_t row, int64_t col, int k, int N,
                                                   int64_t E, FeTerm* out) {
  const int nq = k + 1, nf = k * N + 1, per = nf + N;
  const int64_t nE = E * (int64_t)per;
  const int ent_plus = nq * nq + nq, ent_minus = ent_plus + 1;
  if (row >= nE) {  // a multiplier row: +1 at an in-edge's last flux, -1 at an out-edge's first
    if (col >= nE) return 0;
    const int cp = (int)(col % per);
    if (cp == nf - 1) out[0] = FeTerm{0, ent_plus};
    else if (cp == 0) out[0] = FeTerm{0, ent_minus};
    else return 0;
    return 1;
  }
  const int64_t e = row / per;
  const int pos = (int)(row - e * per);
  const int lc = col >= nE ? -1 : col / per != e ? -2 : (int)(col - e * per);
  return fe_s_terms_loc(pos, lc, k, N, (int)(e * N), out);
}
__host__ __device__ __forceinline__ int fe_s_rhs_terms(int64_t row, int k, int N, int64_t E,
                                                       FeTerm* out) {
  const int nq = k + 1, nf = k * N + 1, per = nf + N;
  const int ent_src = nq * nq + nq + 2, ent_bc = ent_src + 1;
  if (row >= E * (int64_t)per) return 0;
  const int64_t e = row / per;
  const int pos = (int)(row - e * per);
  if (pos >= nf) {
    out[0] = FeTerm{(int)(e * N + pos - nf), ent_src};
    return 1;
  }
  if (pos == 0) out[0] = FeTerm{(int)(2 * e), ent_bc};
  else if (pos == nf - 1) out[0] = FeTerm{(int)(2 * e + 1), ent_bc};
  else return 0;
  return 1;
}

constexpr int kFesWaves = 4;    // k_fe_tasm / k_fe_tres: waves (edges) per block
constexpr int kFesRows = 512;   // (nx_fe_struct_degree) rows per edge: k N + 1 + N + 1 at most
constexpr int kFesCells = 256;  // cells per edge
constexpr int kFesTable = 128;  // term table entries in LDS
// ---- Edge templates (k_fe_tasm / k_fe_tres), any (k, m). An edge's rows (the `per` rows
// from e * per: its flux nodes, then its pressure cells or interior pressure nodes) have the
// same entries on every edge up to a few shapes -- which end has a multiplier column, the
// order of its end nodes' shared rows. nx_create_fe reads each shape's entries from its first
// edge's gather-table terms (cells relative to the edge's first; columns local to the edge,
// or the edge's j-th outside column), checks every other edge's against its shape, and packs
// an entry into 8 bytes; the kernels then form an edge's values and rhs from its R, f, end
// data and cell lengths alone. Same terms in the same order as k_assemble_fe: bit-exact. The
// rows after the edges' (shared node pressures, multipliers) keep the gather tables.
struct FeTplE {
  short lc;       // local column; -(1 + j): the edge's j-th outside column (j < kFeExt)
  short n;        // terms (0..2)
  short c0, c1;   // their cells relative to the edge's first (bc terms: the end, 0 / 1)
  short e0, e1;   // their table entries
};
constexpr int kFeExt = 4;     // outside columns of an edge (multipliers, shared node rows)
constexpr int kFeShapes = 8;  // edge shapes
// An entry packed: x = c0 | c1 << 16, y = e0 | e1 << 7 | n << 14 | (lc + kFeExt) << 16
__host__ __device__ __forceinline__ int2 fe_tpl_pack(const FeTplE& t) {
  return int2{(int)((unsigned)(unsigned short)t.c0 | ((unsigned)(unsigned short)t.c1 << 16)),
              (int)((unsigned)t.e0 | ((unsigned)t.e1 << 7) | ((unsigned)t.n << 14) |
                    ((unsigned)(t.lc + kFeExt) << 16))};
}
struct FeTpl {
  const int2* tpl;     // packed matrix entries, the shapes one after another
  const int2* rtpl;    // packed rhs terms: per shape `per` rows
  const int* rs;       // kFeShapes x (per + 1): each shape's row starts (entry index)
  const int* shape;    // E: the edge's shape
  const int* ext;      // kFeExt E: the edge's outside columns, -1
  const int* rowptr;
  int off[kFeShapes + 1];  // each shape's first entry; off[nsh] = all
  int nsh, per, edge_blocks;
};
constexpr int kFeTplMax = 16384;  // packed entries (LDS: up to 128 KiB)

// one packed term list's value, s = 0 + t0 (+ t1), as fe_term forms them (R: the edge's
// resistance, fe its source, bc its end data, hh its cell lengths)
__device__ __forceinline__ double fe_tpl_val(int2 t, const double* sTv, const int* sKind, double Re,
                                             double fe, const double* bc, const double* hh) {
#pragma clang fp contract(off)
  const int n = (t.y >> 14) & 3;
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (u >= n) break;
    const int e = u ? (t.y >> 7) & 127 : t.y & 127;
    const int c = u ? (int)((unsigned)t.x >> 16) : t.x & 0xffff;
    const double v = sTv[e];
    const int kd = sKind[e];
    s += kd == kFeMass ? (Re * hh[c]) * v
         : kd == kFeSource ? (fe * hh[c]) * v
         : kd == kFeBc ? bc[c] * v
         : v;
  }
  return s;
}

// Dynamic LDS of k_fe_tasm / k_fe_tres (doubles): the packed entries, the rhs terms, the
// row starts, then per wave its edge's cell lengths (and for the residual its x)
size_t fe_tpl_lds(int n_tpl, int nsh, int per, int N, bool res) {
  return 8 * ((size_t)n_tpl + (size_t)nsh * per + ((size_t)kFeShapes * (per + 1) + 1) / 2 +
              (size_t)kFesWaves * (N + (res ? per : 0)));
}

// The templates into LDS, once per workgroup
__device__ __forceinline__ void fe_tpl_stage(const FeTpl& T, int2* sT, int2* sR, int* sRs,
                                             bool rhs) {
  for (int i = threadIdx.x; i < T.off[T.nsh]; i += blockDim.x) sT[i] = T.tpl[i];
  if (rhs)
    for (int i = threadIdx.x; i < T.nsh * T.per; i += blockDim.x) sR[i] = T.rtpl[i];
  for (int i = threadIdx.x; i < kFeShapes * (T.per + 1); i += blockDim.x) sRs[i] = T.rs[i];
}

// Assembly: one wave per edge, the edges in workgroup rounds (the LDS staging amortised); the
// edge's cell lengths loaded once (coalesced), every entry then from LDS alone; values and
// rhs stored coalesced over the edge's contiguous segment and rows. The rows after the
// edges' (shared node pressures, multipliers) from the gather tables, in the blocks after.
__global__ __launch_bounds__(64 * kFesWaves) void k_fe_tasm(FeArgs a, FeTpl T) {
#pragma clang fp contract(off)
  extern __shared__ double fe_lds[];
  __shared__ double sTv[kFesTable];
  __shared__ int sKind[kFesTable];
  const int N = a.N, per = T.per;
  const int64_t E = a.n_edges, nE = E * (int64_t)per;
  if ((int)blockIdx.x >= T.edge_blocks) {
    const int64_t row = nE + (int64_t)(blockIdx.x - T.edge_blocks) * blockDim.x + threadIdx.x;
    if (row >= a.n_rows) return;
    if (a.lhs)
      for (int q = T.rowptr[row]; q < T.rowptr[row + 1]; ++q) {
        double s = 0.0;
        for (int c = a.a_ptr[q]; c < a.a_ptr[q + 1]; ++c) s += fe_term(a, a.a_idx[c], a.a_ent[c]);
        a.val[q] = s;
      }
    if (a.do_rhs) {
      double s = 0.0;
      for (int c = a.b_ptr[row]; c < a.b_ptr[row + 1]; ++c) s += fe_term(a, a.b_idx[c], a.b_ent[c]);
      a.rhs[row] = s;
    }
    return;
  }
  int2* sT = reinterpret_cast<int2*>(fe_lds);
  int2* sR = sT + T.off[T.nsh];
  int* sRs = reinterpret_cast<int*>(sR + T.nsh * per);
  double* sH = reinterpret_cast<double*>(sRs) + (kFeShapes * (per + 1) + 1) / 2;
  for (int i = threadIdx.x; i < kFesTable; i += blockDim.x) {
    sTv[i] = a.tval[i];
    sKind[i] = a.kind[i];
  }
  fe_tpl_stage(T, sT, sR, sRs, a.do_rhs != 0);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double* __restrict__ hh = sH + w * N;
  double* __restrict__ val = a.val;
  double* __restrict__ rhs = a.rhs;
  for (int64_t eb = (int64_t)blockIdx.x * kFesWaves; eb < E; eb += (int64_t)T.edge_blocks * kFesWaves) {
    const int64_t e = eb + w;
    const bool on = e < E;
    __syncthreads();  // (the staging / the previous round's reads of sH)
    if (on)
      for (int c = lane; c < N; c += 64) hh[c] = a.cellh[e * N + c];
    __syncthreads();
    if (!on) continue;
    const int sh = T.shape[e];
    const double Re = a.edge_R[e];
    const double fe = a.edge_f ? a.edge_f[e] : a.f;
    const double bc[2] = {a.edge_bc[2 * e], a.edge_bc[2 * e + 1]};
    if (a.lhs) {
      const int i0 = T.off[sh], L = T.off[sh + 1] - i0;
      const int64_t q0 = T.rowptr[e * per];
      for (int i = lane; i < L; i += 64)
        val[q0 + i] = fe_tpl_val(sT[i0 + i], sTv, sKind, Re, fe, bc, hh);
    }
    if (a.do_rhs) {
      const int2* rt = sR + sh * per;
      for (int r = lane; r < per; r += 64)
        rhs[e * per + r] = fe_tpl_val(rt[r], sTv, sKind, Re, fe, bc, hh);
    }
  }
}

// The true residual r = b - A x with A's edge entries formed again from the templates (the
// CSR's values bit for bit while the coefficients are the assembled ones): one wave per
// edge, its x and cell lengths staged in LDS (coalesced loads), a lane per row summing the
// row's products in CSR order from LDS (its outside columns' x loaded once per edge); the
// rows after the edges' from the CSR in the blocks after. r into rout (a refinement pass
// starts from it); block partials of ||r||^2, ||b||^2 for k_dir_publish.
__global__ __launch_bounds__(64 * kFesWaves) void k_fe_tres(FeArgs a, FeTpl T, Csr A,
                                                             const double* __restrict__ x,
                                                             const double* __restrict__ b,
                                                             double* __restrict__ rout,
                                                             double* __restrict__ partials,
                                                             int nblk) {
#pragma clang fp contract(off)
  extern __shared__ double fe_lds[];
  __shared__ double sTv[kFesTable];
  __shared__ int sKind[kFesTable];
  const int N = a.N, per = T.per;
  const int64_t E = a.n_edges, nE = E * (int64_t)per;
  double rr = 0.0, bb = 0.0;
  if ((int)blockIdx.x >= T.edge_blocks) {
    const int64_t row = nE + (int64_t)(blockIdx.x - T.edge_blocks) * blockDim.x + threadIdx.x;
    if (row < a.n_rows) {
      double s = 0.0;
      for (int q = A.rowptr[row]; q < A.rowptr[row + 1]; ++q) s += A.val[q] * x[A.col[q]];
      const double bv = b[row], rv = bv - s;
      rout[row] = rv;
      rr = rv * rv;
      bb = bv * bv;
    }
  } else {
    int2* sT = reinterpret_cast<int2*>(fe_lds);
    int* sRs = reinterpret_cast<int*>(sT + T.off[T.nsh]);
    double* sH = reinterpret_cast<double*>(sRs) + (kFeShapes * (per + 1) + 1) / 2;
    double* sX = sH + kFesWaves * N;
    for (int i = threadIdx.x; i < kFesTable; i += blockDim.x) {
      sTv[i] = a.tval[i];
      sKind[i] = a.kind[i];
    }
    fe_tpl_stage(T, sT, nullptr, sRs, false);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double* hh = sH + w * N;
    double* xs = sX + w * per;
    for (int64_t eb = (int64_t)blockIdx.x * kFesWaves; eb < E;
         eb += (int64_t)T.edge_blocks * kFesWaves) {
      const int64_t e = eb + w;
      const bool on = e < E;
      __syncthreads();
      if (on) {
        for (int c = lane; c < N; c += 64) hh[c] = a.cellh[e * N + c];
        for (int i = lane; i < per; i += 64) xs[i] = x[e * per + i];
      }
      __syncthreads();
      if (!on) continue;
      const int sh = T.shape[e];
      const int i0 = T.off[sh];
      const int* rs = sRs + sh * (per + 1);
      const double Re = a.edge_R[e];
      const double fe = a.edge_f ? a.edge_f[e] : a.f;
      const double bc[2] = {a.edge_bc[2 * e], a.edge_bc[2 * e + 1]};
      double xo[kFeExt];
#pragma unroll
      for (int j = 0; j < kFeExt; ++j) {
        const int c = T.ext[kFeExt * e + j];
        xo[j] = c >= 0 ? x[c] : 0.0;
      }
      for (int r = lane; r < per; r += 64) {
        double s = 0.0;
        for (int i = rs[r]; i < rs[r + 1]; ++i) {
          const int2 t = sT[i0 + i];
          const int lc = (int)((unsigned)t.y >> 16) - kFeExt;
          double xv = 0.0;
          if (lc >= 0) {
            xv = xs[lc];
          } else {
#pragma unroll
            for (int j = 0; j < kFeExt; ++j)
              if (lc == -1 - j) xv = xo[j];
          }
          s += fe_tpl_val(t, sTv, sKind, Re, fe, bc, hh) * xv;
        }
        const double bv = b[e * per + r], rv = bv - s;
        rout[e * per + r] = rv;
        rr += rv * rv;
        bb += bv * bv;
      }
    }
  }
  block_sum_store(rr, partials + blockIdx.x);
  __syncthreads();
  block_sum_store(bb, partials + nblk + blockIdx.x);
}

// ---- (k, 0) through the condensed P1/DG0 system (nx_fe_set_direct). The divergence against
// DG0 touches a cell's two vertex fluxes only, so the interior fluxes sit in the flux rows
// alone: condensed per cell, the system is P1/DG0's with the cell mass R h [[a, b], [b, a]],
// which the direct tree solve of an auxiliary P1 handle inverts (nx_set_cell_mass).
struct FeCond {
  const double* edge_x;
  const double* edge_R;
  int N, km;  // km = k - 1 interior fluxes per cell
  int64_t E;
  const int *slot, *vfe, *vaux, *ife, *pfe, *paux, *lfe, *laux;
  int nl;
  const double* cst;  // C (2 km) | K (km 2) | Mii (km km)
  double ab;          // a + b
  const double* cellh;  // E*N cell lengths (k_fe_cellh)
};

// The condensed right-hand side b_v - C b_i (vertex rows; pressure and multiplier rows
// copied) into the auxiliary handle's rhs, and (dq_aux) its lumped mass (a + b) R h per cell
// end. One thread per vertex flux, pressure cell, multiplier.
__global__ __launch_bounds__(kBlock) void k_fe_condense(FeCond c, const double* __restrict__ b,
                                                        double* __restrict__ dq_aux,
                                                        double* __restrict__ rhs_aux) {
#pragma clang fp contract(off)
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int N = c.N, km = c.km;
  const int64_t nv = c.E * (N + 1), np = c.E * N;
  if (t < nv) {
    const int64_t e = t / (N + 1);
    const int g = (int)(t - e * (N + 1));
    const double R = c.edge_R[e];
    double bv = b[c.vfe[t]], d = 0.0;
    if (g > 0) {  // the cell on the left: this vertex is its right one (C row 1)
      const int64_t cell = e * N + g - 1;
      d = c.ab * (R * c.cellh[cell]);
      for (int i = 0; i < km; ++i) bv -= c.cst[km + i] * b[c.ife[cell * km + i]];
    }
    if (g < N) {  // the cell on the right: its left vertex (C row 0)
      const int64_t cell = e * N + g;
      d += c.ab * (R * c.cellh[cell]);
      for (int i = 0; i < km; ++i) bv -= c.cst[i] * b[c.ife[cell * km + i]];
    }
    rhs_aux[c.vaux[t]] = bv;
    if (dq_aux) dq_aux[(int64_t)c.slot[e] * (N + 1) + g] = d;
  } else if (t < nv + np) {
    rhs_aux[c.paux[t - nv]] = b[c.pfe[t - nv]];
  } else if (t < nv + np + c.nl) {
    rhs_aux[c.laux[t - nv - np]] = b[c.lfe[t - nv - np]];
  }
}

// The (k, 0) solution from the auxiliary one: vertex fluxes, pressure cells, multipliers
// copied, interior fluxes x_i = Mii b_i / (R h) - K x_v (accum: added, a refinement pass).
__global__ __launch_bounds__(kBlock) void k_fe_expand(FeCond c, const double* __restrict__ xa,
                                                      const double* __restrict__ b,
                                                      double* __restrict__ x, int accum) {
#pragma clang fp contract(off)
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int N = c.N, km = c.km;
  const int64_t nv = c.E * (N + 1), np = c.E * N, n0 = nv + np + c.nl;
  int64_t dst = -1;
  double v = 0.0;
  if (t < nv) {
    dst = c.vfe[t];
    v = xa[c.vaux[t]];
  } else if (t < nv + np) {
    dst = c.pfe[t - nv];
    v = xa[c.paux[t - nv]];
  } else if (t < n0) {
    dst = c.lfe[t - nv - np];
    v = xa[c.laux[t - nv - np]];
  } else if (t < n0 + np) {
    const int64_t cell = t - n0, e = cell / N;
    const int g = (int)(cell - e * N);
    const double Rh = c.edge_R[e] * c.cellh[cell];
    const double xl = xa[c.vaux[e * (N + 1) + g]], xr = xa[c.vaux[e * (N + 1) + g + 1]];
    const double* K = c.cst + 2 * km;
    const double* Mii = c.cst + 4 * km;
    for (int j = 0; j < km; ++j) {
      double s = 0.0;
      for (int i = 0; i < km; ++i) s += Mii[j * km + i] * b[c.ife[cell * km + i]];
      const double xi = s / Rh - K[2 * j] * xl - K[2 * j + 1] * xr;
      const int64_t r = c.ife[cell * km + j];
      x[r] = accum ? x[r] + xi : xi;
    }
    return;
  }
  if (dst >= 0) x[dst] = accum ? x[dst] + v : v;
}

// ---- continuous pressure (k > m >= 1) on a forest: the node-condensed direct solve -------
// (nx_fe_set_cp). Each edge's own unknowns -- its flux nodes and its interior pressure nodes
// -- are eliminated onto its border (p_u, lam_u, p_v, lam_v: the pressure at its end nodes,
// shared with the other edges there, and the multipliers of the bifurcations at its ends).
// Per edge, one thread: every cell's interior nodes condensed onto its two vertices by the
// exact reference blocks (element.condensed_cell_blocks, scaled by s = R h), then the vertices
// (q_i, p_i) eliminated in order along the edge (2 x 2 pivots; the leading blocks of this
// 1-D mixed system are nonsingular) carrying the border columns: the edge's 4 x 4 border
// block Se and rhs ge. The border system over the graph nodes (2 unknowns each: p and lam, lam
// an identity dummy where the node has none) is negative definite and tree-structured: one
// workgroup eliminates it leaf to root by levels and back-substitutes root to leaf. Then each
// edge back-substitutes its vertices and its cells' interiors.
struct CpArgs {
  int N, k, m, nI;
  int64_t E;
  const double* edge_R;
  const double* cellh;
  const double* cst;  // Kh (16) | Ch (4 nI) | Eh (4 nI) | Fh (nI nI)
  const int* tI;      // nI: +1 flux, -1 pressure (interior node types)
  const int* eb;      // per edge: u, v (border node indices), au, av (lam couplings: 0, +-1)
  const int* nrow;    // per border node: its pressure row, its multiplier row (or -1)
  double* fac;        // per vertex (N + 1), per factor (kCpFac), per edge
                      // (edge-minor: a wave's lanes, consecutive edges, touch 512 B per access)
  double* se;         // per edge: Se 16 | ge 4
  double* xn;         // per border node: its (p, lam) values
  const int* gid;     // several ranks: the global edge of each local edge (its se slot)
};
// per vertex (round 6): Pi C 4 | Pi W 8 | Pi rho 2 -- the back-substitution's products
// formed once in the forward sweep (y = Pi rho - (Pi W) x_border - (Pi C) y_next), 14
// doubles instead of Pi | C | W | rho's 18
constexpr int kCpFac = 14;

__device__ __forceinline__ double cp_pow(double s, int ex) {  // s^ex, ex in {-1, 0, 1}
  return ex > 0 ? s : ex < 0 ? 1.0 / s : 1.0;
}
// (the node forest's arithmetic with contraction off: every kernel that inlines it -- the
// lists', the records', the pipelined records' -- rounds the same way, bit for bit)
__device__ __forceinline__ void inv2(const double* P, double* Pi) {
#pragma clang fp contract(off)
  const double det = P[0] * P[3] - P[1] * P[2];
  const double id = 1.0 / det;
  Pi[0] = P[3] * id;
  Pi[1] = -P[1] * id;
  Pi[2] = -P[2] * id;
  Pi[3] = P[0] * id;
}

// The forward sweep of one edge (one thread): Se, ge and the per-vertex factors.
__global__ __launch_bounds__(256) void k_cp_edge(CpArgs a, const double* __restrict__ b) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.E) return;
  const int N = a.N, k = a.k, m = a.m, nI = a.nI;
  const int nf = k * N + 1, per = nf + m * N - 1;
  const int64_t base = e * (int64_t)per;
  const double* bl = b + base;         // this edge's rows of b
  const double* hl = a.cellh + e * N;  // its cells' lengths
  const double* Kh = a.cst;
  const double* Ch = a.cst + 16;
  const int au = a.eb[4 * e + 2], av = a.eb[4 * e + 3];
  const double R = a.edge_R[e];
  double* fe = a.fac + e;
  const int64_t E = a.E;
  auto prow = [&](int j) { return nf + j - 1; };  // interior pressure position j (local row)
  double P[4] = {0.0, 0.0, 0.0, 1.0}, W[8] = {0.0}, rho[2] = {bl[0], 0.0};
  W[1] = (double)au;  // q_0 <-> lam_u
  double Sb[16] = {0.0}, gb[4] = {0.0};
  const int tV[4] = {1, -1, 1, -1};
  for (int c = 0; c < N; ++c) {
    const double s = R * hl[c];
    double K[16];
    for (int r = 0; r < 4; ++r)
      for (int q = 0; q < 4; ++q) K[4 * r + q] = Kh[4 * r + q] * cp_pow(s, (tV[r] + tV[q]) / 2);
    double rV[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = 0; i < nI; ++i) {  // the cell's interior rhs condensed onto its vertices
      const int ti = a.tI[i];
      const double bi = ti > 0 ? bl[c * k + 1 + i] : bl[prow(c * m + 1 + (i - (k - 1)))];
      for (int r = 0; r < 4; ++r) rV[r] -= Ch[r * nI + i] * cp_pow(s, (tV[r] - ti) / 2) * bi;
    }
    double C[4];  // left vertex rows (q, p) x right vertex columns (q, p)
    double Pn[4], Wn[8] = {0.0}, rn[2];
    if (c == 0) {  // the left p is the border p_u
      P[0] += K[0];
      W[0] += K[1];
      Sb[0] += K[5];
      rho[0] += rV[0];
      gb[0] += rV[1];
      C[0] = K[2]; C[1] = K[3]; C[2] = 0.0; C[3] = 0.0;
      Wn[0] = K[9];   // right q <-> p_u
      Wn[4] = K[13];  // right p <-> p_u
    } else {
      P[0] += K[0]; P[1] += K[1]; P[2] += K[4]; P[3] += K[5];
      rho[0] += rV[0];
      rho[1] += rV[1];
      C[0] = K[2]; C[1] = K[3]; C[2] = K[6]; C[3] = K[7];
    }
    if (c + 1 < N) {
      Pn[0] = K[10]; Pn[1] = K[11]; Pn[2] = K[14]; Pn[3] = K[15];
      rn[0] = rV[2] + bl[k * (c + 1)];
      rn[1] = rV[3] + bl[prow(m * (c + 1))];
    } else {  // the right p is the border p_v
      Sb[10] += K[15];
      gb[2] += rV[3];
      if (c == 0) {  // (N = 1: p_u <-> p_v)
        Sb[2] += K[7];
        Sb[8] += K[13];
      }
      Wn[2] += K[11];  // right q <-> p_v
      Wn[3] = (double)av;  // right q <-> lam_v
      Wn[4] = 0.0;  // (the right p slot is a dummy)
      W[2] += C[1];  // left rows <-> p_v
      W[6] += C[3];
      C[1] = 0.0;
      C[3] = 0.0;
      Pn[0] = K[10]; Pn[1] = 0.0; Pn[2] = 0.0; Pn[3] = 1.0;
      rn[0] = rV[2] + bl[nf - 1];
      rn[1] = 0.0;
    }
    double Pi[4];
    inv2(P, Pi);
    // X = Pi C (2 x 2), Y = Pi W (2 x 4), z = Pi rho
    double X[4], Y[8], z[2];
    for (int r = 0; r < 2; ++r) {
      for (int q = 0; q < 2; ++q) X[2 * r + q] = Pi[2 * r] * C[q] + Pi[2 * r + 1] * C[2 + q];
      for (int q = 0; q < 4; ++q) Y[4 * r + q] = Pi[2 * r] * W[q] + Pi[2 * r + 1] * W[4 + q];
      z[r] = Pi[2 * r] * rho[0] + Pi[2 * r + 1] * rho[1];
    }
    for (int r = 0; r < 2; ++r) {  // C^T X, C^T Y, C^T z into the right vertex
      for (int q = 0; q < 2; ++q) Pn[2 * r + q] -= C[r] * X[q] + C[2 + r] * X[2 + q];
      for (int q = 0; q < 4; ++q) Wn[4 * r + q] -= C[r] * Y[q] + C[2 + r] * Y[4 + q];
      rn[r] -= C[r] * z[0] + C[2 + r] * z[1];
    }
    for (int r = 0; r < 4; ++r) {  // W^T Y, W^T z into the border
      for (int q = 0; q < 4; ++q) Sb[4 * r + q] -= W[r] * Y[q] + W[4 + r] * Y[4 + q];
      gb[r] -= W[r] * z[0] + W[4 + r] * z[1];
    }
    double* f = fe + (int64_t)c * kCpFac * E;
    for (int i = 0; i < 4; ++i) f[i * E] = X[i];
    for (int i = 0; i < 8; ++i) f[(4 + i) * E] = Y[i];
    f[12 * E] = z[0];
    f[13 * E] = z[1];
    for (int i = 0; i < 4; ++i) P[i] = Pn[i];
    for (int i = 0; i < 8; ++i) W[i] = Wn[i];
    rho[0] = rn[0];
    rho[1] = rn[1];
  }
  {  // the last vertex
    double Pi[4];
    inv2(P, Pi);
    double Y[8], z[2];
    for (int r = 0; r < 2; ++r) {
      for (int q = 0; q < 4; ++q) Y[4 * r + q] = Pi[2 * r] * W[q] + Pi[2 * r + 1] * W[4 + q];
      z[r] = Pi[2 * r] * rho[0] + Pi[2 * r + 1] * rho[1];
    }
    for (int r = 0; r < 4; ++r) {
      for (int q = 0; q < 4; ++q) Sb[4 * r + q] -= W[r] * Y[q] + W[4 + r] * Y[4 + q];
      gb[r] -= W[r] * z[0] + W[4 + r] * z[1];
    }
    double* f = fe + (int64_t)N * kCpFac * E;
    for (int i = 0; i < 4; ++i) f[i * E] = 0.0;
    for (int i = 0; i < 8; ++i) f[(4 + i) * E] = Y[i];
    f[12 * E] = z[0];
    f[13 * E] = z[1];
  }
  double* o = a.se + 20 * (a.gid ? (int64_t)a.gid[e] : e);
  for (int i = 0; i < 16; ++i) o[i] = Sb[i];
  for (int i = 0; i < 4; ++i) o[16 + i] = gb[i];
}

// The border system over the graph nodes by one workgroup: each node's 2 x 2 block D and rhs
// from its edges (the node's half of their Se / ge) and b at its rows; leaf to root by levels
// P_n = D_n - sum_children B_c^T P_c^-1 B_c (B_c: the child's block of its parent edge, child
// rows x parent columns), then root to leaf x_n = P_n^-1 (h_n - B_n x_parent). Every sum in
// a fixed order (the node's edges / children in list order).
struct CpTree {
  int nn, nlev;
  const int* lev_off;    // nlev + 1: nodes by level, level 0 the roots
  const int* order;      // nodes in level order
  const int* inc_off;    // per node its edges: (edge, end) with end 0 = source, 1 = target
  const int* inc;        // 2 per entry
  const int* parent;     // per node: parent node, the edge to it and this node's end there
  const int* child_off;
  const int* child;
  double* Pinv;  // 4 per node
  double* hv;    // 2 per node
  // per level-order index, the node's record (kCpRec ints, cp_records): every index the
  // node's elimination / back-substitution reads, in one place -- one dependent load instead
  // of the chain order -> offsets -> lists -> entries; nullptr: the lists
  const int* rec;
  // with the records: each node's Schur term for its parent (6 per node: B^T Pc B | B^T Pc h,
  // the expressions cp_up_child_v subtracts), written by the node's own elimination, so the
  // parent reads 6 doubles per child instead of forming them from 10 (round 6)
  double* ctr;
};
// node record (ints): [0] n, [1] pressure row, [2] multiplier row, [3] #edges (-1: more
// than kCpRecInc, read the lists), [4..11] (edge, end) x kCpRecInc, [12] #children (-1: more
// than kCpRecCh), [13..21] (child, its parent edge, its end there) x kCpRecCh, [22] parent,
// [23] parent edge, [24] this node's end of it
constexpr int kCpRecInc = 4, kCpRecCh = 3;
constexpr int kCpRecC = 4 + 2 * kCpRecInc;          // 12: #children
constexpr int kCpRecP = kCpRecC + 1 + 3 * kCpRecCh;  // 22: parent, its edge, this node's end
constexpr int kCpRecPad = 28;                        // (7 x 16 B)
__device__ __forceinline__ void cp_block(const double* se, int e, int ra, int cb, double* B) {
  const double* S = se + 20 * (int64_t)e;  // rows of end ra, columns of end cb (2 x 2)
  B[0] = S[4 * (2 * ra) + 2 * cb];
  B[1] = S[4 * (2 * ra) + 2 * cb + 1];
  B[2] = S[4 * (2 * ra + 1) + 2 * cb];
  B[3] = S[4 * (2 * ra + 1) + 2 * cb + 1];
}
// The node forest's elimination, one node (level order index i): its 2 x 2 pivot block from
// its edges' border blocks minus its children's Schur terms; the pivot's inverse and the
// condensed rhs stored for the back-substitution.
// one incident edge's border block into the node's pivot and rhs
__device__ __forceinline__ void cp_up_edge(const CpArgs& a, int e, int end, double* D, double* g) {
  double B[4];
  cp_block(a.se, e, end, end, B);
  for (int q = 0; q < 4; ++q) D[q] += B[q];
  g[0] += a.se[20 * (int64_t)e + 16 + 2 * end];
  g[1] += a.se[20 * (int64_t)e + 17 + 2 * end];
}
// one child's Schur term, its pivot inverse Pc and rhs hc given
__device__ __forceinline__ void cp_up_child_v(const CpArgs& a, int ce, int cend,
                                              const double* Pc, const double* hc, double* D,
                                              double* g) {
#pragma clang fp contract(off)
  double B[4];  // child rows x this node's columns
  cp_block(a.se, ce, cend, 1 - cend, B);
  double X[4], z[2];  // Pc B, Pc h
  for (int r = 0; r < 2; ++r) {
    for (int q = 0; q < 2; ++q) X[2 * r + q] = Pc[2 * r] * B[q] + Pc[2 * r + 1] * B[2 + q];
    z[r] = Pc[2 * r] * hc[0] + Pc[2 * r + 1] * hc[1];
  }
  for (int r = 0; r < 2; ++r) {
    for (int q = 0; q < 2; ++q) D[2 * r + q] -= B[r] * X[q] + B[2 + r] * X[2 + q];
    g[r] -= B[r] * z[0] + B[2 + r] * z[1];
  }
}
// the node's Schur term for its parent (records' path; the same expressions, the same bits as
// cp_up_child_v forms them in the parent): B = the node's block of its parent edge (node rows
// x parent columns), Pc / hc its pivot inverse and rhs
__device__ __forceinline__ void cp_up_term(const double* B, const double* Pc, const double* hc,
                                           double* o) {
#pragma clang fp contract(off)
  double X[4], z[2];
  for (int r = 0; r < 2; ++r) {
    for (int q = 0; q < 2; ++q) X[2 * r + q] = Pc[2 * r] * B[q] + Pc[2 * r + 1] * B[2 + q];
    z[r] = Pc[2 * r] * hc[0] + Pc[2 * r + 1] * hc[1];
  }
  for (int r = 0; r < 2; ++r) {
    for (int q = 0; q < 2; ++q) o[2 * r + q] = B[r] * X[q] + B[2 + r] * X[2 + q];
    o[4 + r] = B[r] * z[0] + B[2 + r] * z[1];
  }
}
// a child's term into the node's pivot and rhs
__device__ __forceinline__ void cp_up_sub(const double* tc, double* D, double* g) {
  for (int q = 0; q < 4; ++q) D[q] -= tc[q];
  g[0] -= tc[4];
  g[1] -= tc[5];
}
__device__ __forceinline__ void cp_up_child(const CpArgs& a, const CpTree& t, int c, int ce,
                                            int cend, double* D, double* g) {
  cp_up_child_v(a, ce, cend, t.Pinv + 4 * (int64_t)c, t.hv + 2 * (int64_t)c, D, g);
}
__device__ __forceinline__ void cp_node_up(const CpArgs& a, const CpTree& t,
                                           const double* __restrict__ b, int i) {
  double D[4] = {0.0, 0.0, 0.0, 0.0}, g[2];
  int n;
  if (t.rec != nullptr) {  // the record in 7 independent 16-B loads, every index static
    int r[kCpRecPad];
    const int4* q4 = reinterpret_cast<const int4*>(t.rec + (int64_t)kCpRecPad * i);
#pragma unroll
    for (int w = 0; w < kCpRecPad / 4; ++w) {
      const int4 v = q4[w];
      r[4 * w] = v.x;
      r[4 * w + 1] = v.y;
      r[4 * w + 2] = v.z;
      r[4 * w + 3] = v.w;
    }
    n = r[0];
    const int lr = r[2];
    g[0] = b[r[1]];
    g[1] = lr >= 0 ? b[lr] : 0.0;
    if (r[3] >= 0) {
#pragma unroll
      for (int j = 0; j < kCpRecInc; ++j)
        if (j < r[3]) cp_up_edge(a, r[4 + 2 * j], r[5 + 2 * j], D, g);
    } else {
      for (int j = t.inc_off[n]; j < t.inc_off[n + 1]; ++j)
        cp_up_edge(a, t.inc[2 * j], t.inc[2 * j + 1], D, g);
    }
    if (lr < 0) D[3] = 1.0;  // (no multiplier: a decoupled dummy)
    constexpr int kc = kCpRecC;  // the children's part of the record: their terms (ctr)
    if (r[kc] >= 0) {
#pragma unroll
      for (int j = 0; j < kCpRecCh; ++j)
        if (j < r[kc]) cp_up_sub(t.ctr + 6 * (int64_t)r[kc + 1 + 3 * j], D, g);
    } else {
      for (int j = t.child_off[n]; j < t.child_off[n + 1]; ++j)
        cp_up_sub(t.ctr + 6 * (int64_t)t.child[j], D, g);
    }
    double Pi[4];
    inv2(D, Pi);
    for (int q = 0; q < 4; ++q) t.Pinv[4 * (int64_t)n + q] = Pi[q];
    t.hv[2 * n] = g[0];
    t.hv[2 * n + 1] = g[1];
    if (r[kCpRecP] >= 0) {  // this node's term for its parent
      double B[4], o[6];
      cp_block(a.se, r[kCpRecP + 1], r[kCpRecP + 2], 1 - r[kCpRecP + 2], B);
      cp_up_term(B, Pi, g, o);
      for (int q = 0; q < 6; ++q) t.ctr[6 * (int64_t)n + q] = o[q];
    }
    return;
  } else {
    n = t.order[i];
    const int pr = a.nrow[2 * n], lr = a.nrow[2 * n + 1];
    g[0] = b[pr];
    g[1] = lr >= 0 ? b[lr] : 0.0;
    for (int j = t.inc_off[n]; j < t.inc_off[n + 1]; ++j)
      cp_up_edge(a, t.inc[2 * j], t.inc[2 * j + 1], D, g);
    if (lr < 0) D[3] = 1.0;  // (no multiplier: a decoupled dummy)
    for (int j = t.child_off[n]; j < t.child_off[n + 1]; ++j) {
      const int c = t.child[j];
      cp_up_child(a, t, c, t.parent[3 * c + 1], t.parent[3 * c + 2], D, g);
    }
  }
  inv2(D, t.Pinv + 4 * (int64_t)n);
  t.hv[2 * n] = g[0];
  t.hv[2 * n + 1] = g[1];
}
// ... and its back-substitution: the node's values from its parent's
__device__ __forceinline__ void cp_node_down(const CpArgs& a, const CpTree& t, int i) {
#pragma clang fp contract(off)
  int n, p, pe, pend;
  if (t.rec != nullptr) {  // node and parent from the record (one 16-B load each)
    const int* q = t.rec + (int64_t)kCpRecPad * i;
    const int4 h = *reinterpret_cast<const int4*>(q);
    const int4 v = *reinterpret_cast<const int4*>(q + 20);  // [22] parent, [23] its edge
    const int4 w = *reinterpret_cast<const int4*>(q + 24);  // [24] this node's end of it
    n = h.x;
    p = v.z;
    pe = v.w;
    pend = w.x;
  } else {
    n = t.order[i];
    p = t.parent[3 * n];
    pe = t.parent[3 * n + 1];
    pend = t.parent[3 * n + 2];
  }
  double r[2] = {t.hv[2 * n], t.hv[2 * n + 1]};
  if (p >= 0) {
    double B[4];
    cp_block(a.se, pe, pend, 1 - pend, B);
    const double* xp = a.xn + 2 * (int64_t)p;
    r[0] -= B[0] * xp[0] + B[1] * xp[1];
    r[1] -= B[2] * xp[0] + B[3] * xp[1];
  }
  const double* Pn = t.Pinv + 4 * (int64_t)n;
  a.xn[2 * n] = Pn[0] * r[0] + Pn[1] * r[1];
  a.xn[2 * n + 1] = Pn[2] * r[0] + Pn[3] * r[1];
}

// Levels [L0, L1) of the node forest (level 0 the roots) in one workgroup, a barrier per
// level: up = deepest first (the eliminations), else root first (the back-substitution).
// The levels with many nodes run as k_cp_level launches instead (cp_nodes_launch).
__global__ __launch_bounds__(1024) void k_cp_nodes(CpArgs a, CpTree t, const double* __restrict__ b,
                                                   int L0, int L1, int up) {
  for (int k = 0; k < L1 - L0; ++k) {
    const int L = up ? L1 - 1 - k : L0 + k;
    for (int i = t.lev_off[L] + threadIdx.x; i < t.lev_off[L + 1]; i += 1024) {
      if (up) cp_node_up(a, t, b, i);
      else cp_node_down(a, t, i);
    }
    __syncthreads();
  }
}
constexpr int kCpWide = 2048;  // wider levels: grid launches (cp_nodes_launch)

// The same levels with the node records (t.rec), software-pipelined across the level barriers
// (round 6): what a level reads that no level before it writes -- its records, b, its edges'
// border blocks and, going down, its own pivots -- is loaded one level ahead (the record two
// levels ahead going up), so a level waits on one round trip (its children's pivots and rhs
// going up, its parent's values going down) instead of three. Same arithmetic, same order as
// cp_node_up / cp_node_down. Levels of at most 1024 nodes (one per thread) whose records all
// hold their node's edges and children (cp_lev_full; else the level-by-level kernels).
struct CpUpMid {
  int i, n, nch;  // i < 0: no node
  double D[4], g[2];
  int ch[kCpRecCh];
  int pe, pend;  // the parent edge and this node's end of it (pe < 0: a root)
};
__device__ __forceinline__ void cp_rec_load(const CpTree& t, int i, int (&r)[kCpRecPad]) {
  if (i < 0) return;
  const int4* q4 = reinterpret_cast<const int4*>(t.rec + (int64_t)kCpRecPad * i);
#pragma unroll
  for (int w = 0; w < kCpRecPad / 4; ++w) {
    const int4 v = q4[w];
    r[4 * w] = v.x;
    r[4 * w + 1] = v.y;
    r[4 * w + 2] = v.z;
    r[4 * w + 3] = v.w;
  }
}
// a level's part that no level before it writes: b, its edges' border blocks (one level ahead)
__device__ __forceinline__ void cp_up_mid(const CpArgs& a, const double* __restrict__ b, int i,
                                          const int (&r)[kCpRecPad], CpUpMid& m) {
  constexpr int kc = kCpRecC;
  m.i = i;
  m.nch = 0;
  m.pe = -1;
  if (i < 0) return;
  m.n = r[0];
#pragma unroll
  for (int q = 0; q < 4; ++q) m.D[q] = 0.0;
  const int lr = r[2];
  m.g[0] = b[r[1]];
  m.g[1] = lr >= 0 ? b[lr] : 0.0;
#pragma unroll
  for (int j = 0; j < kCpRecInc; ++j)
    if (j < r[3]) cp_up_edge(a, r[4 + 2 * j], r[5 + 2 * j], m.D, m.g);
  if (lr < 0) m.D[3] = 1.0;
  m.nch = r[kc];
#pragma unroll
  for (int j = 0; j < kCpRecCh; ++j) m.ch[j] = r[kc + 1 + 3 * j];
  if (r[kCpRecP] >= 0) {
    m.pe = r[kCpRecP + 1];
    m.pend = r[kCpRecP + 2];
  }
}
// ... and the part after the level below: its children's terms (loaded first thing in the
// level, with its own parent block: one round trip), the pivot, its term for its parent
struct CpUpIn {
  double tc[kCpRecCh][6], B[4];
};
__device__ __forceinline__ void cp_up_in(const CpArgs& a, const CpTree& t, const CpUpMid& m,
                                         CpUpIn& in) {
  if (m.i < 0) return;
#pragma unroll
  for (int j = 0; j < kCpRecCh; ++j)
    if (j < m.nch)
#pragma unroll
      for (int q = 0; q < 6; ++q) in.tc[j][q] = t.ctr[6 * (int64_t)m.ch[j] + q];
  if (m.pe >= 0) cp_block(a.se, m.pe, m.pend, 1 - m.pend, in.B);
}
__device__ __forceinline__ void cp_up_fin(const CpArgs& a, const CpTree& t,
                                          const double* __restrict__ b, CpUpMid& m,
                                          const CpUpIn& in) {
  if (m.i < 0) return;
#pragma unroll
  for (int j = 0; j < kCpRecCh; ++j)
    if (j < m.nch) cp_up_sub(in.tc[j], m.D, m.g);
  double Pi[4];
  inv2(m.D, Pi);
#pragma unroll
  for (int q = 0; q < 4; ++q) t.Pinv[4 * (int64_t)m.n + q] = Pi[q];
  t.hv[2 * m.n] = m.g[0];
  t.hv[2 * m.n + 1] = m.g[1];
  if (m.pe >= 0) {
    double o[6];
    cp_up_term(in.B, Pi, m.g, o);
#pragma unroll
    for (int q = 0; q < 6; ++q) t.ctr[6 * (int64_t)m.n + q] = o[q];
  }
}
struct CpDnMid {
  int n, p;  // n < 0: no node
  double r[2], B[4], P[4];
};
__device__ __forceinline__ void cp_dn_rec(const CpTree& t, int i, int4 (&r)[3]) {
  if (i < 0) return;
  const int* q = t.rec + (int64_t)kCpRecPad * i;
  r[0] = *reinterpret_cast<const int4*>(q);
  r[1] = *reinterpret_cast<const int4*>(q + 20);  // [22] parent, [23] its edge
  r[2] = *reinterpret_cast<const int4*>(q + 24);  // [24] this node's end of it
}
__device__ __forceinline__ void cp_dn_mid(const CpArgs& a, const CpTree& t, int i,
                                          const int4 (&r)[3], CpDnMid& m) {
  m.n = -1;
  if (i < 0) return;
  const int n = r[0].x, p = r[1].z, pe = r[1].w, pend = r[2].x;
  m.n = n;
  m.p = p;
  m.r[0] = t.hv[2 * n];
  m.r[1] = t.hv[2 * n + 1];
  if (p >= 0) cp_block(a.se, pe, pend, 1 - pend, m.B);
#pragma unroll
  for (int q = 0; q < 4; ++q) m.P[q] = t.Pinv[4 * (int64_t)n + q];
}
__device__ __forceinline__ void cp_dn_fin(const CpArgs& a, CpDnMid& m) {
#pragma clang fp contract(off)
  if (m.n < 0) return;
  double r0 = m.r[0], r1 = m.r[1];
  if (m.p >= 0) {
    const double* xp = a.xn + 2 * (int64_t)m.p;
    r0 -= m.B[0] * xp[0] + m.B[1] * xp[1];
    r1 -= m.B[2] * xp[0] + m.B[3] * xp[1];
  }
  a.xn[2 * m.n] = m.P[0] * r0 + m.P[1] * r1;
  a.xn[2 * m.n + 1] = m.P[2] * r0 + m.P[3] * r1;
}
constexpr int kCpPipeLv = 64;  // levels per k_cp_nodes_rec launch (their ranges in LDS)
constexpr int kCpChunk = 128;  // nodes per level of a subtree chunk (its workgroup's threads)
// rng: a run of wide levels in subtree chunks, one per workgroup (each level's [start, end)
// of this chunk; nx_fe_set_cp), or nullptr: levels [L0, L1) whole, in one workgroup
__global__ __launch_bounds__(1024) void k_cp_nodes_rec(CpArgs a, CpTree t,
                                                       const double* __restrict__ b,
                                                       const int* __restrict__ rng, int L0,
                                                       int L1, int up) {
  __shared__ int sLo[kCpPipeLv], sHi[kCpPipeLv];
  const int nlv = L1 - L0;
  for (int k = threadIdx.x; k < nlv; k += blockDim.x) {
    if (rng != nullptr) {
      sLo[k] = rng[2 * ((int64_t)blockIdx.x * nlv + k)];
      sHi[k] = rng[2 * ((int64_t)blockIdx.x * nlv + k) + 1];
    } else {
      sLo[k] = t.lev_off[L0 + k];
      sHi[k] = t.lev_off[L0 + k + 1];
    }
  }
  __syncthreads();
  // the node of this thread at the pass's k-th level (-1: none)
  auto node = [&](int k) {
    if (k >= nlv) return -1;
    const int L = up ? nlv - 1 - k : k;
    const int i = sLo[L] + (int)threadIdx.x;
    return i < sHi[L] ? i : -1;
  };
  if (up) {
    int r[kCpRecPad];
    CpUpMid m, mn;
    int i = node(0);
    cp_rec_load(t, i, r);
    cp_up_mid(a, b, i, r, m);
    int inx = node(1);
    cp_rec_load(t, inx, r);  // level 1's record
    for (int k = 0; k < nlv; ++k) {
      CpUpIn in;
      cp_up_in(a, t, m, in);        // level k: its children's terms (the one wait)
      cp_up_mid(a, b, inx, r, mn);  // level k + 1: b and its border blocks
      inx = node(k + 2);
      cp_rec_load(t, inx, r);       // level k + 2: its record
      cp_up_fin(a, t, b, m, in);
      __syncthreads();
      m = mn;
    }
  } else {
    int4 r[3];
    CpDnMid m, mn;
    int i = node(0);
    cp_dn_rec(t, i, r);
    cp_dn_mid(a, t, i, r, m);
    int inx = node(1);
    cp_dn_rec(t, inx, r);
    for (int k = 0; k < nlv; ++k) {
      cp_dn_mid(a, t, inx, r, mn);  // level k + 1: its pivots, rhs and parent blocks
      inx = node(k + 2);
      cp_dn_rec(t, inx, r);
      cp_dn_fin(a, m);              // level k: the parent's values (the one wait)
      __syncthreads();
      m = mn;
    }
  }
}

// One level [i0, i1) of level-order nodes, a thread per node across the grid
__global__ __launch_bounds__(256) void k_cp_level(CpArgs a, CpTree t, const double* __restrict__ b,
                                                  int i0, int i1, int up) {
  const int i = i0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= i1) return;
  if (up) cp_node_up(a, t, b, i);
  else cp_node_down(a, t, i);
}

// Back-substitution of one edge (one thread): its vertices from the border values, then every
// cell's interior nodes; x written (accum: added -- a refinement pass), the node rows too by
// the edges whose source they are (or, for a node no edge leaves, its first edge in).
// xs: dynamic LDS for the workgroup's edges' rows of x (blockDim.x * per doubles), written
// out unit-stride at the end (round 6: lane-strided row stores left partial lines, 1.67x
// the algorithmic traffic); nullptr-sized launch (0 bytes): the rows stored directly.
__global__ __launch_bounds__(256) void k_cp_back(CpArgs a, const double* __restrict__ b,
                                                 double* __restrict__ x, const int* __restrict__ nown,
                                                 int accum, int stage) {
  extern __shared__ double cp_xs[];
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int N = a.N, k = a.k, m = a.m, nI = a.nI;
  const int nf = k * N + 1, per = nf + m * N - 1;
  const int64_t base = e * (int64_t)per;
  if (e < a.E) {
  const double* bl = b + base;         // this edge's rows of b
  const double* hl = a.cellh + e * N;  // its cells' lengths
  const int u = a.eb[4 * e], v = a.eb[4 * e + 1];
  const double xb[4] = {a.xn[2 * u], a.xn[2 * u + 1], a.xn[2 * v], a.xn[2 * v + 1]};
  const double* fe = a.fac + e;
  const int64_t E = a.E;
  const double* Eh = a.cst + 16 + 4 * nI;
  const double* Fh = Eh + 4 * nI;
  const double R = a.edge_R[e];
  auto put = [&](int64_t r, double val) { x[r] = accum ? x[r] + val : val; };
  auto putl = [&](int r, double val) {  // the edge's local row r
    if (stage)
      cp_xs[(int64_t)threadIdx.x * per + r] = val;
    else
      put(base + r, val);
  };
  auto prow = [&](int j) { return nf + j - 1; };  // (local row)
  double yn[2] = {0.0, 0.0};  // the next vertex's (q, p)
  const int tV[4] = {1, -1, 1, -1};
  // (the vertex factors one vertex ahead: the next vertex's loads fly while this one computes)
  double fv[kCpFac], fn[kCpFac];
#pragma unroll
  for (int q = 0; q < kCpFac; ++q) fn[q] = fe[((int64_t)N * kCpFac + q) * E];
  for (int i = N; i >= 0; --i) {
#pragma unroll
    for (int q = 0; q < kCpFac; ++q) fv[q] = fn[q];
    if (i > 0) {
      const double* f = fe + (int64_t)(i - 1) * kCpFac * E;
#pragma unroll
      for (int q = 0; q < kCpFac; ++q) fn[q] = f[q * E];
    }
    double y0 = fv[12], y1 = fv[13];
    for (int q = 0; q < 4; ++q) {
      y0 -= fv[4 + q] * xb[q];
      y1 -= fv[8 + q] * xb[q];
    }
    y0 -= fv[0] * yn[0] + fv[1] * yn[1];
    y1 -= fv[2] * yn[0] + fv[3] * yn[1];
    putl(k * i, y0);
    if (i > 0 && i < N) putl(prow(m * i), y1);
    if (i < N) {  // cell i: its interior nodes from (q_i, p_i, q_{i+1}, p_{i+1})
      const double s = R * hl[i];
      const double xv[4] = {y0, i == 0 ? xb[0] : y1, yn[0], i + 1 == N ? xb[2] : yn[1]};
      for (int j = 0; j < nI; ++j) {
        const int tj = a.tI[j];
        double val = 0.0;
        for (int l = 0; l < nI; ++l) {
          const int tl = a.tI[l];
          const double bv = tl > 0 ? bl[i * k + 1 + l] : bl[prow(i * m + 1 + (l - (k - 1)))];
          val += Fh[j * nI + l] * cp_pow(s, -(tj + tl) / 2) * bv;
        }
        for (int q = 0; q < 4; ++q) val -= Eh[j * 4 + q] * cp_pow(s, (-tj + tV[q]) / 2) * xv[q];
        putl(tj > 0 ? i * k + 1 + j : prow(i * m + 1 + (j - (k - 1))), val);
      }
    }
    yn[0] = y0;
    yn[1] = y1;
  }
  // the border rows: node values written once (the node's designated edge, nown)
  for (int end = 0; end < 2; ++end) {
    const int n = end ? v : u;
    if (nown[n] != e) continue;
    put(a.nrow[2 * n], a.xn[2 * n]);
    if (a.nrow[2 * n + 1] >= 0) put(a.nrow[2 * n + 1], a.xn[2 * n + 1]);
  }
  }  // e < a.E
  if (stage) {  // the workgroup's edge rows out, unit stride (every row of an edge written)
    __syncthreads();
    const int T = blockDim.x;
    const int64_t e0 = (int64_t)blockIdx.x * T;
    const int ne = (int)min<int64_t>(T, a.E - e0);
    double* gx = x + e0 * per;
    for (int j = threadIdx.x; j < ne * per; j += T) gx[j] = accum ? gx[j] + cp_xs[j] : cp_xs[j];
  }
}

// Several ranks: the node rows' rhs this rank owns into the summed node rhs (2 per node)
__global__ __launch_bounds__(256) void k_cp_nb(const int* __restrict__ nrowx, int nn,
                                               const double* __restrict__ b,
                                               double* __restrict__ nb) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= 2 * nn) return;
  const int r = nrowx[i];
  if (r >= 0) nb[i] = b[r];
}

// The edge templates (FeTpl) of a layout with `per` rows per edge: each shape's entries and
// rhs terms from its first edge's gather-table terms, every other edge's checked against its
// shape (row lengths, local / outside columns, terms); false (the gather kernels stay) on any
// difference, more than kFeShapes shapes or kFeExt outside columns, or fields out of range.
struct FeTplBuild {
  std::vector<int> ent, rent;  // per edge entry: packed lc / terms (for the comparison)
  std::vector<FeTplE> t, r;
  std::vector<int> rs;
};
bool fe_term_rel(const int32_t* kind, int ent, int idx, int64_t e, int N, short& c) {
  const int kd = kind[ent];
  if (kd == kFeMass || kd == kFeSource) {
    const int64_t rel = idx - e * N;
    if (rel < 0 || rel >= N) return false;
    c = (short)rel;
  } else if (kd == kFeBc) {
    const int64_t rel = idx - 2 * e;
    if (rel < 0 || rel > 1) return false;
    c = (short)rel;
  } else {
    c = 0;
  }
  return ent >= 0 && ent < 128;
}
bool fe_build_tpl(nx_network* h, int per, int32_t N, int64_t E, int64_t n_rows,
                  const int32_t* rowptr, const int32_t* col, const int32_t* kind,
                  const int32_t* a_ptr, const int32_t* a_idx, const int32_t* a_ent,
                  const int32_t* b_ptr, const int32_t* b_idx, const int32_t* b_ent) {
  const int64_t nE = E * (int64_t)per;
  if (per < 1 || per >= 32767 || N >= 32767 || nE > n_rows || N > kFesCells) return false;
  std::vector<FeTplE> shp_t[kFeShapes], shp_r[kFeShapes];
  std::vector<int> shp_rs[kFeShapes];
  int nsh = 0;
  std::vector<int> shape((size_t)E), ext((size_t)kFeExt * E, -1);
  std::vector<FeTplE> et, er;
  std::vector<int> ers(per + 1);
  auto same = [](const FeTplE& x, const FeTplE& y) {
    return x.lc == y.lc && x.n == y.n && x.c0 == y.c0 && x.c1 == y.c1 && x.e0 == y.e0 &&
           x.e1 == y.e1;
  };
  for (int64_t e = 0; e < E; ++e) {
    const int64_t r0 = e * per;
    et.clear();
    er.clear();
    int ne = 0;
    int* xe = ext.data() + (size_t)kFeExt * e;
    for (int pos = 0; pos < per; ++pos) {
      ers[pos] = (int)et.size();
      for (int q = rowptr[r0 + pos]; q < rowptr[r0 + pos + 1]; ++q) {
        const int64_t cq = col[q];
        FeTplE x{};
        if (cq >= r0 && cq < r0 + per) {
          x.lc = (short)(cq - r0);
        } else {
          int j = 0;
          while (j < ne && xe[j] != cq) ++j;
          if (j == ne) {
            if (ne == kFeExt) return false;
            xe[ne++] = (int)cq;
          }
          x.lc = (short)(-1 - j);
        }
        const int n = a_ptr[q + 1] - a_ptr[q];
        if (n < 1 || n > 2) return false;
        x.n = (short)n;
        if (!fe_term_rel(kind, a_ent[a_ptr[q]], a_idx[a_ptr[q]], e, N, x.c0)) return false;
        x.e0 = (short)a_ent[a_ptr[q]];
        if (n > 1) {
          if (!fe_term_rel(kind, a_ent[a_ptr[q] + 1], a_idx[a_ptr[q] + 1], e, N, x.c1)) return false;
          x.e1 = (short)a_ent[a_ptr[q] + 1];
        }
        et.push_back(x);
      }
      const int nr = b_ptr[r0 + pos + 1] - b_ptr[r0 + pos];
      if (nr > 2) return false;
      FeTplE y{};
      y.n = (short)nr;
      if (nr > 0) {
        if (!fe_term_rel(kind, b_ent[b_ptr[r0 + pos]], b_idx[b_ptr[r0 + pos]], e, N, y.c0)) return false;
        y.e0 = (short)b_ent[b_ptr[r0 + pos]];
      }
      if (nr > 1) {
        if (!fe_term_rel(kind, b_ent[b_ptr[r0 + pos] + 1], b_idx[b_ptr[r0 + pos] + 1], e, N, y.c1))
          return false;
        y.e1 = (short)b_ent[b_ptr[r0 + pos] + 1];
      }
      er.push_back(y);
    }
    ers[per] = (int)et.size();
    int sh = 0;
    for (; sh < nsh; ++sh) {
      if (shp_t[sh].size() != et.size() || shp_rs[sh] != ers) continue;
      bool eq = true;
      for (size_t i = 0; i < et.size() && eq; ++i) eq = same(shp_t[sh][i], et[i]);
      for (int i = 0; i < per && eq; ++i) eq = same(shp_r[sh][i], er[i]);
      if (eq) break;
    }
    if (sh == nsh) {
      if (nsh == kFeShapes) return false;
      shp_t[nsh] = et;
      shp_r[nsh] = er;
      shp_rs[nsh] = ers;
      ++nsh;
    }
    shape[e] = sh;
  }
  std::vector<int2> packed, rpacked;
  std::vector<int> rs_all((size_t)kFeShapes * (per + 1), 0);
  int off[kFeShapes + 1] = {};
  for (int sh = 0; sh < nsh; ++sh) {
    off[sh] = (int)packed.size();
    for (const FeTplE& x : shp_t[sh]) packed.push_back(fe_tpl_pack(x));
    for (const FeTplE& y : shp_r[sh]) rpacked.push_back(fe_tpl_pack(y));
    std::copy(shp_rs[sh].begin(), shp_rs[sh].end(), rs_all.begin() + (size_t)sh * (per + 1));
  }
  off[nsh] = (int)packed.size();
  if (packed.empty() || off[nsh] > kFeTplMax) return false;
  if (fe_tpl_lds(off[nsh], nsh, per, N, true) > 150 * 1024) return false;  // (+ static LDS)
  for (int i = 0; i <= nsh; ++i) h->fe_tpl_off[i] = off[i];
  h->fe_tpl_nsh = nsh;
  h->fe_tpl_per = per;
  if (upload(&h->fe_tpl_buf, packed.data(), (int64_t)packed.size(), h->stream) ||
      upload(&h->fe_tpl_rbuf, rpacked.data(), (int64_t)rpacked.size(), h->stream) ||
      upload(&h->fe_tpl_rs, rs_all.data(), (int64_t)rs_all.size(), h->stream) ||
      upload(&h->fe_tpl_shape, shape.data(), E, h->stream) ||
      upload(&h->fe_tpl_lam, ext.data(), (int64_t)ext.size(), h->stream) ||
      hipStreamSynchronize(h->stream) != hipSuccess)
    return false;
  return true;
}
// rows per edge of the layouts nx_create_fe may be given: flux degree k, pressure degree m
// (DG0 for m = 0), by the size of the term table; the first whose templates check out
bool fe_try_tpl(nx_network* h, int32_t N, int64_t E, int64_t n_rows, int32_t n_table,
                const int32_t* rowptr, const int32_t* col, const int32_t* kind,
                const int32_t* a_ptr, const int32_t* a_idx, const int32_t* a_ent,
                const int32_t* b_ptr, const int32_t* b_idx, const int32_t* b_ent) {
  for (int k = 1; k <= 16; ++k)
    for (int m = 0; m < k || (m == 0 && k == 1); ++m) {
      const int npl = m == 0 ? 1 : m + 1;
      if (n_table != (k + 1) * (k + 1) + npl * (k + 1) + 2 + npl + 1) continue;
      const int per = k * N + 1 + (m == 0 ? N : m * N - 1);
      if (E * (int64_t)per > n_rows) continue;
      if (fe_build_tpl(h, per, N, E, n_rows, rowptr, col, kind, a_ptr, a_idx, a_ent, b_ptr,
                       b_idx, b_ent))
        return true;
    }
  return false;
}
int fe_per(const nx_network* h) { return h->fe_tpl_per; }
bool fe_tpl_on(const nx_network* h) {
  const char* e = std::getenv("NXHIP_FE_STRUCT");  // read per launch: tests switch it
  return h->fe_tpl && (e == nullptr || std::atoi(e) != 0);
}
FeTpl fe_tpl_args(const nx_network* h, int edge_blocks) {
  FeTpl t{h->fe_tpl_buf, h->fe_tpl_rbuf, h->fe_tpl_rs, h->fe_tpl_shape, h->fe_tpl_lam, h->rowptr,
          {}, h->fe_tpl_nsh, h->fe_tpl_per, edge_blocks};
  for (int i = 0; i <= kFeShapes; ++i) t.off[i] = h->fe_tpl_off[i];
  return t;
}
void opt_in_lds(const void* fn, int bytes);
// the dynamic LDS of the template kernels (opted in past 64 KiB: high degrees, long edges)
size_t fe_tpl_lds_of(const nx_network* h, bool res) {
  const size_t b = fe_tpl_lds(h->fe_tpl_off[h->fe_tpl_nsh], h->fe_tpl_nsh, h->fe_tpl_per,
                              (int)h->N, res);
  if (b > 64 * 1024)
    opt_in_lds(res ? reinterpret_cast<const void*>(&k_fe_tres)
                   : reinterpret_cast<const void*>(&k_fe_tasm), 150 * 1024);
  return b;
}
// edge workgroups of the template kernels: rounds of kFesWaves edges, a few per CU
int fe_tpl_blocks(const nx_network* h) {
  return std::max(1, std::min(grid_of(h->E, kFesWaves), 8 * h->n_cu));
}

// terms [ptr[i], ptr[i+1]) of every output i must reference the table and the cell / edge
// arrays in range
int check_terms(const char* what, int64_t n_out, const int32_t* ptr, const int32_t* idx,
                const int32_t* ent, int32_t n_table, const int32_t* kind, int64_t n_cells,
                int64_t n_edges) {
  if (ptr[0] != 0) return fail(NX_ERR_ARG, std::string(what) + ": ptr[0] must be 0");
  for (int64_t i = 0; i < n_out; ++i)
    if (ptr[i + 1] < ptr[i]) return fail(NX_ERR_ARG, std::string(what) + ": ptr not monotone");
  for (int64_t t = 0; t < ptr[n_out]; ++t) {
    if (ent[t] < 0 || ent[t] >= n_table)
      return fail(NX_ERR_ARG, std::string(what) + ": table entry out of range");
    const int k = kind[ent[t]];
    const int64_t lim = (k == kFeMass || k == kFeSource) ? n_cells : k == kFeBc ? 2 * n_edges : 1;
    if (k != kFeConst && (idx[t] < 0 || idx[t] >= lim))
      return fail(NX_ERR_ARG, std::string(what) + ": term index out of range");
  }
  return NX_OK;
}

// The flux degree k when the tables are exactly a (k, 0) layout's (fe_s_terms generates every
// entry's and every rhs row's term list, compared entry by entry), else 0 (the gather kernel).
int fe_struct_degree(int32_t N, int64_t E, int64_t n_rows, const int32_t* rowptr,
                     const int32_t* col, int32_t n_table, const int32_t* a_ptr,
                     const int32_t* a_idx, const int32_t* a_ent, const int32_t* b_ptr,
                     const int32_t* b_idx, const int32_t* b_ent) {
  int k = 0;
  for (int kk = 1; kk <= 16 && !k; ++kk)
    if (n_table == (kk + 1) * (kk + 1) + (kk + 1) + 4 &&
        n_rows >= E * (int64_t)(kk * N + 1 + N))
      k = kk;
  if (!k || k * N + 1 + N + 1 > kFesRows || N > kFesCells || n_table > kFesTable)
    return 0;  // (the template sizes)
  FeTerm t[2];
  for (int64_t r = 0; r < n_rows; ++r) {
    for (int q = rowptr[r]; q < rowptr[r + 1]; ++q) {
      const int n = fe_s_terms(r, col[q], k, N, E, t);
      if (n == 0 || a_ptr[q + 1] - a_ptr[q] != n) return 0;
      for (int u = 0; u < n; ++u)
        if (a_idx[a_ptr[q] + u] != t[u].idx || a_ent[a_ptr[q] + u] != t[u].ent) return 0;
    }
    const int n = fe_s_rhs_terms(r, k, N, E, t);
    if (b_ptr[r + 1] - b_ptr[r] != n) return 0;
    for (int u = 0; u < n; ++u)
      if (b_idx[b_ptr[r] + u] != t[u].idx || b_ent[b_ptr[r] + u] != t[u].ent) return 0;
  }
  return k;
}

}  // namespace

NX_API int nx_fe_struct_degree(int32_t N, int64_t n_edges, int64_t n_rows, const int32_t* rowptr,
                               const int32_t* col, int32_t n_table, const int32_t* a_ptr,
                               const int32_t* a_idx, const int32_t* a_ent, const int32_t* b_ptr,
                               const int32_t* b_idx, const int32_t* b_ent, int32_t* k_out) {
  if (!rowptr || !col || !a_ptr || !a_idx || !a_ent || !b_ptr || !b_idx || !b_ent || !k_out)
    return fail(NX_ERR_ARG, "NULL array");
  if (N < 1 || n_edges < 1 || n_rows < 1) return fail(NX_ERR_ARG, "bad sizes");
  *k_out = fe_struct_degree(N, n_edges, n_rows, rowptr, col, n_table, a_ptr, a_idx, a_ent,
                            b_ptr, b_idx, b_ent);
  return NX_OK;
}

NX_API int nx_create_fe(int32_t device, int32_t N, int64_t n_edges, const double* edge_x,
                        int64_t n_rows, const int32_t* rowptr, const int32_t* col,
                        int64_t n_ghost, int32_t n_table, const int32_t* table_kind,
                        const double* table_val,
                        const int32_t* a_ptr, const int32_t* a_idx, const int32_t* a_ent,
                        const int32_t* b_ptr, const int32_t* b_idx, const int32_t* b_ent,
                        nx_network_t** out) {
  if (out == nullptr) return fail(NX_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (N < 1 || n_edges < 1 || n_rows < 1 || n_table < 1 || n_ghost < 0)
    return fail(NX_ERR_ARG, "N, n_edges, n_rows and n_table must be >= 1, n_ghost >= 0");
  if (!edge_x || !rowptr || !col || !table_kind || !table_val || !a_ptr || !a_idx || !a_ent ||
      !b_ptr || !b_idx || !b_ent)
    return fail(NX_ERR_ARG, "NULL array");
  for (int32_t i = 0; i < n_table; ++i)
    if (table_kind[i] < kFeConst || table_kind[i] > kFeBc)
      return fail(NX_ERR_ARG, "table_kind must be 0..3");
  if (rowptr[0] != 0) return fail(NX_ERR_ARG, "rowptr[0] must be 0");
  const int64_t nnz = rowptr[n_rows];
  const int64_t n_cells = n_edges * (int64_t)N;
  if (n_cells >= (int64_t)INT32_MAX) return fail(NX_ERR_ARG, "too many cells for 32-bit terms");
  CHECK(check_terms("matrix terms", nnz, a_ptr, a_idx, a_ent, n_table, table_kind, n_cells,
                    n_edges));
  CHECK(check_terms("rhs terms", n_rows, b_ptr, b_idx, b_ent, n_table, table_kind, n_cells,
                    n_edges));
  // the CSR pattern rides on nx_create's host-given row path (no graph edges): it validates
  // the pattern and allocates the solver; the edge data and term tables are added here
  std::vector<double> zeros((size_t)std::max<int64_t>(nnz, 1), 0.0);
  nx_network_t* h = nullptr;
  CHECK(nx_create(device, N, 0, nullptr, nullptr, n_rows, rowptr, col, zeros.data(), n_ghost,
                  &h));
  h->fe = true;
  h->E = n_edges;
  int rc = NX_OK;
  if ((rc = upload(&h->edge_x, edge_x, 6 * n_edges, h->stream)) ||
      (rc = dalloc(&h->edge_R, n_edges)) || (rc = dalloc(&h->edge_bc, 2 * n_edges)) ||
      (rc = upload(&h->fe_kind, table_kind, (int64_t)n_table, h->stream)) ||
      (rc = upload(&h->fe_tval, table_val, (int64_t)n_table, h->stream)) ||
      (rc = upload(&h->fe_aptr, a_ptr, nnz + 1, h->stream)) ||
      (rc = upload(&h->fe_aidx, a_idx, (int64_t)a_ptr[nnz], h->stream)) ||
      (rc = upload(&h->fe_aent, a_ent, (int64_t)a_ptr[nnz], h->stream)) ||
      (rc = upload(&h->fe_bptr, b_ptr, n_rows + 1, h->stream)) ||
      (rc = upload(&h->fe_bidx, b_idx, (int64_t)b_ptr[n_rows], h->stream)) ||
      (rc = upload(&h->fe_bent, b_ent, (int64_t)b_ptr[n_rows], h->stream)) ||
      (rc = dalloc(&h->fe_cellh, n_cells)) ||
      hipStreamSynchronize(h->stream) != hipSuccess) {
    nx_destroy(h);
    return rc ? rc : fail(NX_ERR_HIP, "upload of the element tables failed");
  }
  hipLaunchKernelGGL(k_fe_cellh, dim3(grid_of(n_cells, kBlock)), dim3(kBlock), 0, h->stream,
                     h->edge_x, (int)N, n_cells, h->fe_cellh);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(h->stream) != hipSuccess) {
    nx_destroy(h);
    return fail(NX_ERR_HIP, "cell lengths failed");
  }
  // (a rank layout's ghost columns are outside both analyses: the gather tables run it)
  h->fe_sk = n_ghost ? 0 : fe_struct_degree(N, n_edges, n_rows, rowptr, col, n_table, a_ptr,
                                            a_idx, a_ent, b_ptr, b_idx, b_ent);
  h->fe_tpl = n_ghost ? false : fe_try_tpl(h, N, n_edges, n_rows, n_table, rowptr, col,
                                           table_kind, a_ptr, a_idx, a_ent, b_ptr, b_idx, b_ent);
  *out = h;
  return NX_OK;
}

namespace {
void xr_free(nx_network* h);
int xr_alloc(nx_network* h, int P);
int xr_link(nx_network* h, const std::vector<XPeer>& peers);
XPeer xpeer_of(void* base, int P);
}  // namespace

NX_API int nx_fe_templates(nx_network_t* h, int32_t* n_shapes, int32_t* rows_per_edge) {
  if (!h || !n_shapes || !rows_per_edge) return fail(NX_ERR_ARG, "null argument");
  *n_shapes = h->fe_tpl ? h->fe_tpl_nsh : 0;
  *rows_per_edge = h->fe_tpl ? h->fe_tpl_per : 0;
  return NX_OK;
}

NX_API int nx_destroy(nx_network_t* h) {
  if (h) h->pend_lhs = h->pend_rhs = 0;  // nothing to assemble for a dying handle
  if (h == nullptr) return NX_OK;
  if (h->group) return fail(NX_ERR_STATE, "destroy the group (nx_group_destroy) first");
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  xr_free(h);
  {
    nx_network* hs[1] = {h};
    (void)drop_graph(graph_slot(Team{hs, 1, nullptr}));
  }
  if (h->comm) ncclCommDestroy(h->comm);
  hc_close(h->hcomm);
  h->hcomm = nullptr;
  if (h->d_agree) (void)hipFree(h->d_agree);
  void* bufs[] = {h->edge_x, h->edge_lm, h->edge_seg, h->edge_R, h->edge_bc, h->edge_f, h->lm_val, h->dq,
                  h->z, h->vv, h->vs, h->hist,
                  h->rowptr, h->col,     h->val,      h->rhs,    h->vb[0],   h->vb[1],
                  h->wb[0],  h->wb[1],   h->x,        h->tmp,    h->partials, h->st,
                  h->partA,  h->partB,   h->red,
                  h->send_idx, h->send_buf, h->gath, h->d_seq,
                  h->fe_kind, h->fe_tval, h->fe_aptr, h->fe_aidx, h->fe_aent,
                  h->fe_bptr, h->fe_bidx, h->fe_bent, h->out_idx,
                  h->d_left_k, h->d_cut_own, h->d_gk_off, h->d_gk_row, h->d_gk_coef, h->cutbuf,
                  h->d_cyc_rows, h->cyc_z, h->cyc_cinv, h->cyc_cap, h->cyc_prev, h->cyc_w,
                  h->fe_slot, h->fe_vfe, h->fe_vaux, h->fe_ife, h->fe_pfe, h->fe_paux, h->fe_lfe,
                  h->fe_laux, h->fe_cst, h->fe_cellh, h->d_cyc_qloc, h->d_cyc_lcol, h->cyc_u,
                  h->cp_cst, h->cp_fac, h->cp_se, h->cp_xn, h->cp_Pinv, h->cp_hv, h->cp_ctr, h->cp_tI,
                  h->cp_eb, h->cp_nrow, h->cp_lev_off, h->cp_order, h->cp_inc_off, h->cp_inc,
                  h->cp_parent, h->cp_child_off, h->cp_child, h->cp_nown, h->cp_gid,
                  h->cp_nrowx, h->cp_rec, h->cp_rng, h->fe_tpl_buf,
                  h->fe_tpl_rbuf, h->fe_tpl_rs, h->fe_tpl_shape, h->fe_tpl_lam};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  for (void* p : h->pc_bufs)
    if (p) (void)hipFree(p);
  if (h->h_st) (void)hipHostFree(h->h_st);
  if (h->h_last) (void)hipHostFree(h->h_last);
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : h->ev_pool)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : h->dev)
    if (e) (void)hipEventDestroy(e);
  for (double* p : h->snap)
    if (p) (void)hipFree(p);
  for (auto& e : h->snap_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : h->fe_ev)
    if (e) (void)hipEventDestroy(e);
  if (h->copy_stream) (void)hipStreamDestroy(h->copy_stream);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return NX_OK;
}

NX_API int nx_dims(nx_network_t* h, int64_t* n_rows, int64_t* n_cols, int64_t* nnz) {
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (n_rows) *n_rows = h->n_own;
  if (n_cols) *n_cols = h->n_col;
  if (nnz) *nnz = h->nnz;
  return NX_OK;
}

namespace {
int chain_rec_refresh(nx_network* h);
}  // namespace

NX_API int nx_set_coefficients(nx_network_t* h, const double* edge_R, double R_const, double f,
                               const double* edge_bc) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (h->E > 0 && edge_bc == nullptr) return fail(NX_ERR_ARG, "edge_bc is NULL");
  CHECK(set_device(h));
  if (h->E > 0) {
    if (edge_R) {
      HIPCALL(hipMemcpyAsync(h->edge_R, edge_R, sizeof(double) * h->E, hipMemcpyHostToDevice,
                             h->stream));
    } else {
      std::vector<double> Rc((size_t)h->E, R_const);
      HIPCALL(hipMemcpyAsync(h->edge_R, Rc.data(), sizeof(double) * h->E, hipMemcpyHostToDevice,
                             h->stream));
      HIPCALL(hipStreamSynchronize(h->stream));
    }
    HIPCALL(hipMemcpyAsync(h->edge_bc, edge_bc, sizeof(double) * 2 * h->E, hipMemcpyHostToDevice,
                           h->stream));
  }
  h->f = f;
  h->have_coeffs = true;
  h->coef_version += 1;  // (R may have changed: the next lhs assembly is a new matrix)
  HIPCALL(hipStreamSynchronize(h->stream));
  return chain_rec_refresh(h);
}

NX_API int nx_set_source(nx_network_t* h, const double* edge_f) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  CHECK(set_device(h));
  if (edge_f == nullptr) {
    if (h->edge_f) HIPCALL(hipFree(h->edge_f));
    h->edge_f = nullptr;
    return chain_rec_refresh(h);
  }
  if (h->E > 0) {
    if (!h->edge_f) CHECK(dalloc(&h->edge_f, h->E));
    HIPCALL(hipMemcpyAsync(h->edge_f, edge_f, sizeof(double) * h->E, hipMemcpyHostToDevice,
                           h->stream));
    HIPCALL(hipStreamSynchronize(h->stream));
  }
  return chain_rec_refresh(h);
}

namespace {

// Launch the assembly kernel (values and / or rhs; the lumped mass dq with the values unless
// dq says otherwise) on stream s (the handle's by default).
int launch_assembly(nx_network* h, int lhs, int rhs, int dq = -1, hipStream_t s = nullptr) {
  if (!s) s = h->stream;
  if (dq < 0) dq = lhs;
  if (dq) h->dq_stale = false;
  if (h->fe) {  // general degrees: one thread per nonzero / rhs row
    FeArgs a{h->edge_x, h->edge_R, h->edge_bc, h->f, h->edge_f, h->N, h->fe_kind, h->fe_tval,
             h->fe_aptr, h->fe_aidx, h->fe_aent, h->fe_bptr, h->fe_bidx, h->fe_bent,
             h->nnz, h->n_own, h->val, h->rhs, lhs, rhs, h->E, h->fe_cellh};
    hipEvent_t e0 = h->prof ? h->ev[0] : nullptr, e1 = h->prof ? h->ev[1] : nullptr;
    // (k, 0): the edge templates (NXHIP_FE_STRUCT=0: the gather tables), else the tables
    if (fe_tpl_on(h)) {
      const int eb = fe_tpl_blocks(h);
      const int lb = (int)grid_of(h->n_own - h->E * (int64_t)fe_per(h), 64 * kFesWaves);
      hipExtLaunchKernelGGL(k_fe_tasm, dim3(eb + lb), dim3(64 * kFesWaves),
                            fe_tpl_lds_of(h, false), s, e0, e1, 0, a, fe_tpl_args(h, eb));
    } else {
      hipExtLaunchKernelGGL(k_assemble_fe, dim3(grid_of(std::max(h->nnz, h->n_own), kBlock)),
                            dim3(kBlock), 0, s, e0, e1, 0, a);
    }
    HIPCALL(hipGetLastError());
    return NX_OK;
  }
  // one launch: edge blocks (4 edges each) then the multiplier-row blocks
  const int64_t nlm = std::max(h->nnz_lm, h->B);
  // edges per wave: 4 for N < 16, 2 for N < 32, else 1 (k_assemble, 64-cell chunks)
  const int epw = h->N < 16 ? 4 : h->N < 32 ? 2 : 1;
  const int eb = grid_of(grid_of(h->E, epw), kBlock / 64);
  const int lb = grid_of(nlm, kBlock);
  if (eb + lb > 0) {
    AsmArgs a{EdgeArgs{h->edge_x, h->edge_lm, h->edge_seg, h->E, h->N},
              h->edge_R, h->edge_bc, h->f, h->edge_f, h->val, h->rhs, dq ? h->dq : nullptr, lhs, rhs,
              eb, h->nnz_lm, h->B, h->lm_val, h->val + h->nnz_edges, h->rhs + h->n_edge_dofs};
    hipEvent_t e0 = h->prof ? h->ev[0] : nullptr, e1 = h->prof ? h->ev[1] : nullptr;
    if (epw == 4)
      hipExtLaunchKernelGGL(k_assemble_seg<16>, dim3(eb + lb), dim3(kBlock), 0, s, e0, e1, 0, a);
    else if (epw == 2)
      hipExtLaunchKernelGGL(k_assemble_seg<32>, dim3(eb + lb), dim3(kBlock), 0, s, e0, e1, 0, a);
    else
      hipExtLaunchKernelGGL(k_assemble, dim3(eb + lb), dim3(kBlock), 0, s, e0, e1, 0, a);
  }
  HIPCALL(hipGetLastError());
  return NX_OK;
}

// Deferred assembly: on one rank (no group, no communicator, P1/DG0) nx_assemble only
// records what to assemble, and the next call that uses the device -- every NX_API entry
// point flushes it first -- launches it; the direct solve captures it as the head of its
// own graph instead (one launch per step less).
bool defer_ok(const nx_network* h) { return !h->fe; }

// The lumped flux mass before a reader of dq (a refinement pass, the separate sweeps, MINRES,
// the graph path) when the last assembly was a one-launch step's, which does not form it:
// the assembly kernel's dq-only launch (the same arithmetic and order: the same bits). Eager,
// outside any captured graph.
int ensure_dq(nx_network* h) {
  if (!h->dq_stale) return NX_OK;
  return launch_assembly(h, 0, 0, 1);
}

int flush_assembly(nx_network* h) {
  if (!h || !(h->pend_lhs || h->pend_rhs)) return NX_OK;
  const int lhs = h->pend_lhs, rhs = h->pend_rhs;
  h->pend_lhs = h->pend_rhs = 0;
  CHECK(set_device(h));
  CHECK(launch_assembly(h, lhs, rhs));
  if (h->prof && (h->E > 0 || h->fe)) {  // profiling: the assembly kernel's own events
    HIPCALL(hipEventSynchronize(h->ev[1]));
    float ms = 0.f;
    HIPCALL(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    h->asm_ms += ms;
    h->asm_cnt += 1;
  }
  return NX_OK;
}

}  // namespace

namespace {
// k_dir_step's chain records from the edge arrays (decomposition or coefficients changed)
int chain_rec_refresh(nx_network* h) {
  if (!h->d_crec || h->E == 0) return NX_OK;
  hipLaunchKernelGGL(k_chain_rec, dim3(grid_of(h->E, 256)), dim3(256), 0, h->stream,
                     h->pa.chain_edge, h->pa.chain_flip, h->E, h->edge_x, h->edge_R, h->edge_f,
                     h->f, h->edge_bc, h->edge_lm, h->edge_seg, h->d_crec, h->d_ci);
  HIPCALL(hipGetLastError());
  HIPCALL(hipStreamSynchronize(h->stream));
  return NX_OK;
}
// the tile width W of a (W, CPL) variant (nx_set_preconditioner's choice)
int variant_w(int v) { return v == 5 || v == 7 || v == 10 ? 8 : v == 6 ? 4 : v <= 2 ? 16 : 64; }
int variant_cpl(int v) {
  return v == 0 ? 1 : (v == 1 || v == 3 || v == 5) ? 2 : v == 10 ? 3 : v == 8 ? 8 : v == 9 ? 16 : 4;
}
}  // namespace

NX_API int nx_assemble(nx_network_t* h, int32_t lhs, int32_t rhs) {
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (!h->have_coeffs) return fail(NX_ERR_STATE, "nx_set_coefficients must be called first");
  if (!lhs && !rhs) return NX_OK;
  if (defer_ok(h)) {
    h->pend_lhs |= lhs ? 1 : 0;
    h->pend_rhs |= rhs ? 1 : 0;
  } else {
    CHECK(flush_assembly(h));
    CHECK(set_device(h));
    CHECK(launch_assembly(h, lhs, rhs));
    if (h->prof && h->E > 0) {
      HIPCALL(hipEventSynchronize(h->ev[1]));
      float ms = 0.f;
      HIPCALL(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
      h->asm_ms += ms;
      h->asm_cnt += 1;
    }
  }
  if (lhs) {
    h->have_lhs = true;
    // a graph with cycles rebuilds its Woodbury correction (2 n_cyc tree solves) only when
    // the matrix values can have changed: new coefficients since the last lhs assembly
    if (h->asm_coef_version != h->coef_version) {
      h->lhs_version += 1;
      h->asm_coef_version = h->coef_version;
    }
  }
  if (rhs) h->have_rhs = true;
  return NX_OK;
}

namespace {

// ---- single rank with the preconditioner: the whole solve is one graph launch in the
// common case. Head graph = start application z = P^{-1} b (condensed straight from the
// rhs; its down sweep also builds the factored coefficients and G), then k_mr_a(1) (which
// initialises the state from beta_1^2), then (preconditioner k, k_mr_a(k+1)) for k = 1..L-1. It ends with
// k_mr_a(L), L even, so S[0] holds the latest state; the exact preconditioner converges
// in 3 iterations and k_mr_a(4) applies the last update. Continuation chunks (rarely
// needed) are (preconditioner k, k_mr_a(k+1)) for L consecutive k.
void launch_a_lean(nx_network* h, int64_t k, bool init, double rtol, int maxit,
                   const double* r1in = nullptr, bool mark = false) {
  double* r1 = h->vb[(k - 1) & 1];
  MrVecs mv{r1,    r1in ? r1in : r1, h->vb[k & 1], h->wb[k & 1], h->wb[(k - 1) & 1],
            h->x,  h->z,             h->vv,        h->vs,        h->n_own,         h->hist};
  const MrInit ini{init ? 1 : 0, nB_of(h), maxit, rtol, h->partB, mark ? 1 : 0, h->d_seq, h->d_last};
  hipLaunchKernelGGL((k_mr_a<false, true>), dim3(h->nA), dim3(kBlock), 0, h->stream, csr_of(h), mv,
                     h->st + ((k + 1) & 1), h->st + (k & 1), h->partB, nB_of(h), h->red, h->partA,
                     h->chunksA, ini);
}

int launch_head_lean(nx_network* h, int L, double rtol, int maxit) {
  // start: mode 1 only reads y, so it condenses the rhs itself; with the LDS kernels its
  // down sweep also computes the factored coefficients and G (k_pc_down_lds, mode 1)
  launch_pc<false>(h, h->rhs, h->rhs, h->st, h->st + 1, 1, 0);
  launch_pc<false>(h, h->rhs, h->rhs, h->st, h->st + 1, 1, 1);
  if (!h->pc_lds) {
    const bool fac = h->pa.dc_kappa != nullptr;
    const int ncols = h->pa.dense ? h->pa.n_top : 0;
    const int nmax = (int)std::max<int64_t>(h->pc_ndc, h->pc_slots);
    const int grid = std::max(ncols, std::max(1, grid_of(nmax, 64)));
    hipLaunchKernelGGL(k_pc_prep, dim3(grid), dim3(64), 0, h->stream, h->pa, fac ? (int)h->pc_ndc : 0,
                       fac ? (int)h->pc_slots : 0, ncols, nullptr, nullptr, (int64_t)0);
  }
  launch_a_lean(h, 1, true, rtol, maxit);
  // iteration 1 reads r_1 = b straight from the rhs (no copy): as r2 in the preconditioner
  // of k = 1 and as r_{k-1} in k_mr_a(2)
  for (int k = 1; k < L; ++k) {
    double* y = h->vb[(k - 1) & 1];
    const double* r2 = k == 1 ? h->rhs : h->vb[k & 1];
    MrState* st = h->st + (k & 1);
    MrState* other = h->st + ((k + 1) & 1);
    launch_pc<false>(h, y, r2, st, other, 0, 0);
    launch_pc<false>(h, y, r2, st, other, 0, 1);
    launch_a_lean(h, k + 1, false, rtol, maxit, k == 1 ? h->rhs : nullptr, k + 1 == L);
  }
  HIPCALL(hipGetLastError());
  return NX_OK;
}

// Wait for the state published by the last k_mr_a of the graph just launched (sequence
// number h->seq). Spins on host-coherent memory; checks the stream now and then so a
// failed launch cannot hang the host.
int wait_published(nx_network* h) {
  const int want = h->seq;
  for (uint64_t spin = 1;; ++spin) {
    if (__atomic_load_n(&h->h_last->pad, __ATOMIC_ACQUIRE) == want) return NX_OK;
    // (a stream query now and then -- about every millisecond -- catches a launch that ended
    // without publishing; more often, one could land on the publish and delay seeing it)
    if ((spin & 16383) == 0) {
      const hipError_t e = hipStreamQuery(h->stream);
      if (e == hipSuccess) {  // stream idle: the stamp must be there now
        if (__atomic_load_n(&h->h_last->pad, __ATOMIC_ACQUIRE) == want) return NX_OK;
        return fail(NX_ERR_STATE, "solve graph finished without publishing its state");
      }
      if (e != hipErrorNotReady) return fail(NX_ERR_HIP, std::string("solve graph: ") +
                                                             hipGetErrorString(e));
    }
  }
}

int capture(nx_network* h, hipGraph_t* graph, hipGraphExec_t* exec,
            const std::function<int()>& body) {
  HIPCALL(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
  const int rc = body();
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(h->stream, &g);
  if (rc != NX_OK) {
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  if (e != hipSuccess) return fail(NX_ERR_HIP, std::string("capture: ") + hipGetErrorString(e));
  *graph = g;
  HIPCALL(hipGraphInstantiate(exec, g, nullptr, nullptr, 0));
  return NX_OK;
}

// ---- several ranks (RCCL, one process per GPU; or an in-process group) with the
// preconditioner: the same one-graph solve. Head = the start application from the rhs
// (ghost slots of the rhs and of r are zero from allocation and stay zero) with its coarse
// all-reduce, the per-solve coefficients (or the fused start), iterations 1..L-1, then the
// halo and k_mr_a of iteration L (published). beta_1^2 travels with the halo of iteration 1 like every later
// beta^2 (point-to-point gather), so k_mr_a(1) initialises the state itself.
int launch_head_multi(const Team& t, int L, double rtol, int maxit) {
  CHECK(team_pc(t, 0, 1, true));
  for (int r = 0; r < t.P; ++r) {  // coefficients of this assembly's D (fixed per solve)
    nx_network* h = t.hs[r];
    if (h->pc_lds && h->pa.fused && h->pc_jobs > 0) continue;  // the start's down sweep did it
    if (h->pa.dc_kappa) {
      const int nmax = (int)std::max<int64_t>(h->pc_ndc, h->pc_slots);
      if (nmax > 0)
        hipLaunchKernelGGL(k_pc_factor, dim3(grid_of(nmax, 256)), dim3(256), 0, h->stream, h->pa,
                           (int)h->pc_ndc, (int)h->pc_slots);
    }
    if (h->pa.mdense) {
      hipLaunchKernelGGL(k_pc_gbuild, dim3(h->pa.n_top), dim3(64), 0, h->stream, h->pa);
      hipLaunchKernelGGL(k_pc_wroot, dim3(1), dim3(kTopThreads), 0, h->stream, h->pa);
    }
  }
  const LeanOpt first{true, L == 1, rtol, maxit};
  CHECK(launch_part_a(t, 1, &first));
  for (int k = 1; k < L; ++k) {
    CHECK(launch_part_pc(t, k, true));
    const LeanOpt next{false, k + 1 == L, rtol, maxit};
    CHECK(launch_part_a(t, k + 1, &next));
  }
  HIPCALL(hipGetLastError());
  return NX_OK;
}

LeanGraphs& lean_of(const Team& t) { return t.g ? t.g->lean : t.hs[0]->lean; }

// ---- direct tree solve (k_dir_*): y in vb[1], w in vb[0], S^{-1} w in z, x
// refine = 0: x = A^{-1} b; refine = 1: one step of iterative refinement, x += A^{-1} r with
// r = b - A x as the previous pass's residual check left it in tmp. Both end with the true
// residual (r kept in tmp again) published.

// One rank, direct: the top part in every down workgroup (pa.topdown) -- only when the jobs
// run in one round (every workgroup repeats the top part; C4 on one GPU, 4 rounds, measured
// 0.524 vs 0.488 ms/step with the top kernel)
// (an auxiliary solve of the (k, 0) route too: no residual check, workgroup 0 writes x's top
// values itself)
bool top_down_on(const nx_network* h) {
  return (h->fres_ok || h->cond_mass) && h->top_nt > 0 && h->pc_jobs <= h->n_cu;
}

template <int W, int CPL>
void launch_direct_wc(nx_network* h, double rtol, int refine, bool prof) {
  const hipEvent_t* evs = prof ? h->dev : nullptr;
  if (refine && h->need_r) {  // the fused step (k_dir_step) kept no residual: r = b - A x
    const int nrb = grid_of(h->n_own, kRowsPerBlock * res_chunks(h->n_own));
    hipLaunchKernelGGL(k_residual_ck, dim3(nrb), dim3(kBlock), 0, h->stream, csr_of(h), h->x,
                       h->rhs, h->partials, nrb, h->tmp, res_chunks(h->n_own));
    h->need_r = false;
  }
  // refine: the previous pass's residual check left r = b - A x in tmp
  const double* bin = refine ? h->tmp : h->rhs;
  const bool cyc = h->n_cyc > 0 && !h->cyc_raw;  // graphs with cycles: Woodbury after the sweeps
  const int m = 2 * h->n_cyc;
  if (cyc && refine)  // U^T x before the sweeps add the tree solve's correction
    hipLaunchKernelGGL(k_cyc_w, dim3(grid_of(m, 256)), dim3(256), sizeof(double) * m, h->stream, h->x, h->d_cyc_rows, m,
                       h->cyc_cinv, nullptr, h->cyc_w, h->cyc_prev);
  {  // the LDS sweeps in mode kModeDirect (direct_local: pc_lds)
    h->pa.accum = refine ? 1 : 0;  // refinement: the sweeps add the correction to x
    h->pa.fres = h->fres_ok ? 1 : 0;  // and the down sweep the residual check
    // and every down workgroup the top part (no k_pc_top_lds) when the jobs run in one round
    const bool td = top_down_on(h);
    h->pa.topdown = td ? 1 : 0;
    launch_pc<false>(h, const_cast<double*>(bin), bin, h->st, h->st + 1, kModeDirect, 0, h->x, evs);
    launch_pc<false>(h, const_cast<double*>(bin), bin, h->st, h->st + 1, kModeDirect, 1, h->x, evs);
    h->pa.accum = 0;
    h->pa.fres = 0;
    h->pa.topdown = 0;
    if (h->fres_ok) {
      const int ntop = td ? h->top_nt : 0;
      hipExtLaunchKernelGGL(k_dir_publish_fr, dim3(1), dim3(kReduceThreads), 0, h->stream,
                            prof ? h->dev[6] : nullptr, prof ? h->dev[7] : nullptr, 0, h->pa.rpart,
                            h->pc_jobs, h->d_left, h->n_left, csr_of(h), h->x, h->rhs, h->tmp,
                            h->dir_bb, refine, rtol, h->d_seq, h->d_last,
                            h->pa.slot_lam + h->top_ts0, h->pa.slot_z + h->top_ts0, ntop);
      return;
    }
  }
  if (h->cond_mass) return;  // an auxiliary solve: the (k, 0) handle checks its own residual
  if (cyc) {  // x -= Z Cinv U^T (x - x_before): the couplings the tree solve dropped
    hipLaunchKernelGGL(k_cyc_w, dim3(grid_of(m, 256)), dim3(256), sizeof(double) * m, h->stream, h->x, h->d_cyc_rows, m,
                       h->cyc_cinv, refine ? h->cyc_prev : nullptr, h->cyc_w, nullptr);
    hipLaunchKernelGGL(k_cyc_fix, dim3(grid_of(h->n_own, kBlock)), dim3(kBlock), 0, h->stream,
                       h->x, h->cyc_z, h->n_col, h->cyc_w, m, h->n_own);
  }
  const int nrb = grid_of(h->n_own, kRowsPerBlock * res_chunks(h->n_own));
  hipExtLaunchKernelGGL(k_residual_ck, dim3(nrb), dim3(kBlock), 0, h->stream,
                        prof ? h->dev[6] : nullptr, prof ? h->dev[7] : nullptr, 0, csr_of(h), h->x,
                        h->rhs, h->partials, nrb, h->tmp, res_chunks(h->n_own));  // r kept: refinement
  hipLaunchKernelGGL(k_dir_publish, dim3(1), dim3(kReduceThreads), 0, h->stream, h->partials,
                     nrb, rtol, h->d_seq, h->d_last);
}

// The fused direct step (k_dir_step): one rank, the deferred assembly pending, the LDS
// sweeps with the fused residual, one round of jobs (all resident), direct launches (a graph
// would freeze the launch count), not disabled by a failed launch or NXHIP_DIR_FUSED=0.
bool dstep_on(const nx_network* h) {
  const char* e = std::getenv("NXHIP_DIR_FUSED");  // read per solve: tests switch it
  const bool env = e == nullptr || std::atoi(e) != 0;
  return env && h->dstep_ok && !h->dstep_off && h->pc_lds && h->fres_ok && h->pa.exact &&
         h->pc_jobs > 0 && h->pc_jobs <= h->n_cu && !proc_rank(h) && h->group == nullptr &&
         h->nranks == 1;
}

DirStep dir_args(nx_network* h, double rtol);
template <int CPL>
bool sup_launch(const DirStep& da);
template <int W, int CPL>
void launch_dstep_wc(nx_network* h, double rtol, bool prof) {
  const DirStep da = dir_args(h, rtol);
  static thread_local std::vector<const void*> opted;  // (the dynamic LDS above 64 KiB, once)
  const bool sup = sup_launch<CPL>(da);
  h->last_sup = sup;
  const void* fn = sup ? reinterpret_cast<const void*>(&k_dir_step<W, CPL, CPL <= 2>)
                       : reinterpret_cast<const void*>(&k_dir_step<W, CPL>);
  if (std::find(opted.begin(), opted.end(), fn) == opted.end()) {
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kDirLdsMax);
    (void)hipGetLastError();
    opted.push_back(fn);
  }
  if (sup)
    hipExtLaunchKernelGGL((k_dir_step<W, CPL, CPL <= 2>), dim3(h->pc_jobs), dim3(kPcThreads),
                          h->dstep_lds, h->stream, prof ? h->dev[0] : nullptr,
                          prof ? h->dev[1] : nullptr, 0, h->pa, da);
  else
    hipExtLaunchKernelGGL((k_dir_step<W, CPL>), dim3(h->pc_jobs), dim3(kPcThreads), h->dstep_lds,
                          h->stream, prof ? h->dev[0] : nullptr, prof ? h->dev[1] : nullptr, 0,
                          h->pa, da);
}

// Several ranks: k_dir_team_up, the assembly + up sweep + top part of one rank (half 0 of
// launch_direct_team's first pass; pa.accum / fres / coarsedown as the caller set them).
template <int W, int CPL>
void launch_dteam_wc(nx_network* h) {
  DirStep da{h->edge_x, h->edge_R, h->edge_bc, h->edge_f, h->f, h->edge_lm, h->edge_seg,
             h->val, h->rhs, h->dq, h->nnz_lm, h->B, h->lm_val, h->val + h->nnz_edges,
             h->rhs + h->n_edge_dofs, h->x, nullptr, nullptr, 0, nullptr, h->d_tsync, 0, 0,
             0.0, 0, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL((k_dir_team_up<W, CPL>), dim3(h->pc_jobs), dim3(kPcThreads), 0, h->stream,
                     h->pa, da);
}
void launch_dteam(nx_network* h) {
  switch (h->pc_variant) {
    case 0: launch_dteam_wc<16, 1>(h); break;
    case 1: launch_dteam_wc<16, 2>(h); break;
    case 2: launch_dteam_wc<16, 4>(h); break;
    case 3: launch_dteam_wc<64, 2>(h); break;
    case 5: launch_dteam_wc<8, 2>(h); break;
    case 7: launch_dteam_wc<8, 4>(h); break;
    case 8: launch_dteam_wc<64, 8>(h); break;
    case 9: launch_dteam_wc<64, 16>(h); break;
    default: launch_dteam_wc<64, 4>(h); break;
  }
}
// k_dir_team_up applies: the LDS sweeps with a top part (every rank's coarse junctions are
// top slots), the fused residual, the counter, one pending assembly of values and rhs.
bool dteam_on(const nx_network* h) {
  const char* e = std::getenv("NXHIP_DIR_FUSED");  // read per solve: tests switch it
  const bool env = e == nullptr || std::atoi(e) != 0;
  return env && h->pc_lds && h->fres_ok && h->d_tsync && h->pc_jobs > 0 && h->top_nt > 0 &&
         h->top_nt <= kTopThreads && h->pa.n_top_lvl <= kMaxTopLvl && !h->fe;
}

// Launch k_dir_step and wait for its published state (the host's sequence advances).
int run_dstep(nx_network* h, double rtol, bool prof) {
  switch (h->dstep_variant) {
    case 0: launch_dstep_wc<16, 1>(h, rtol, prof); break;
    case 1: launch_dstep_wc<16, 2>(h, rtol, prof); break;
    case 2: launch_dstep_wc<16, 4>(h, rtol, prof); break;
    case 3: launch_dstep_wc<64, 2>(h, rtol, prof); break;
    case 5: launch_dstep_wc<8, 2>(h, rtol, prof); break;
    case 7: launch_dstep_wc<8, 4>(h, rtol, prof); break;
    case 10: launch_dstep_wc<8, 3>(h, rtol, prof); break;
    default: launch_dstep_wc<64, 4>(h, rtol, prof); break;
  }
  HIPCALL(hipGetLastError());
  h->dstep_epoch += 1;
  h->seq += 1;
  return wait_published(h);
}

int launch_direct(nx_network* h, double rtol, int refine, bool prof = false) {
  switch (h->pc_variant) {
    case 0: launch_direct_wc<16, 1>(h, rtol, refine, prof); break;
    case 1: launch_direct_wc<16, 2>(h, rtol, refine, prof); break;
    case 2: launch_direct_wc<16, 4>(h, rtol, refine, prof); break;
    case 3: launch_direct_wc<64, 2>(h, rtol, refine, prof); break;
    case 5: launch_direct_wc<8, 2>(h, rtol, refine, prof); break;
    case 6: launch_direct_wc<4, 4>(h, rtol, refine, prof); break;
    case 7: launch_direct_wc<8, 4>(h, rtol, refine, prof); break;
    case 8: launch_direct_wc<64, 8>(h, rtol, refine, prof); break;
    case 9: launch_direct_wc<64, 16>(h, rtol, refine, prof); break;
    default: launch_direct_wc<64, 4>(h, rtol, refine, prof); break;
  }
  HIPCALL(hipGetLastError());
  return NX_OK;
}

// Cinv = (C^{-1} + U^T Z)^{-1} from cyc_cap (m x m U^T Z, then the m / 2 couplings a) on the
// device: Gauss-Jordan with partial pivoting (k_gj_*), 2 m launches on the handle's stream,
// stored transposed for the correction's kernels; the same on every rank of a team (the same
// summed inputs, the same operations). One host sync: a zero coupling or pivot fails loudly.
int cyc_invert(nx_network* h) {
  const int m = 2 * h->n_cyc;
  if (!h->cyc_gj) HIPCALL(hipMalloc((void**)&h->cyc_gj, sizeof(double) * 2 * (size_t)m * m + 8));
  int* bad = reinterpret_cast<int*>(h->cyc_gj + 2 * (size_t)m * m);
  HIPCALL(hipMemsetAsync(bad, 0, sizeof(int), h->stream));
  const int gb = std::min(4096, grid_of(2 * (int64_t)m * m, 256));
  hipLaunchKernelGGL(k_gj_init, dim3(gb), dim3(256), 0, h->stream, h->cyc_cap, m, h->cyc_gj, bad);
  for (int col = 0; col < m; ++col) {
    hipLaunchKernelGGL(k_gj_pivot, dim3(1), dim3(1024), 0, h->stream, h->cyc_gj, m, col, bad);
    hipLaunchKernelGGL(k_gj_elim, dim3(m), dim3(256), 0, h->stream, h->cyc_gj, m, col);
  }
  hipLaunchKernelGGL(k_gj_out, dim3(std::min(4096, grid_of((int64_t)m * m, 256))), dim3(256), 0,
                     h->stream, h->cyc_gj, m, h->cyc_cinv);
  HIPCALL(hipGetLastError());
  int b = 0;
  HIPCALL(hipMemcpyAsync(&b, bad, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  HIPCALL(hipStreamSynchronize(h->stream));
  if (b == 1) return fail(NX_ERR_STATE, "cycle chain: no coupling at its grounded end");
  if (b == 2) return fail(NX_ERR_STATE, "cycle correction is singular");
  return NX_OK;
}

// Graphs with cycles: Z = A_g^{-1} U column by column (the tree solve of a unit right-hand
// side, accumulated into a zeroed x), then C^{-1} + U^T Z inverted on the host (m <= 256,
// Gauss-Jordan with partial pivoting). Once per assembled matrix.
int cyc_build(nx_network* h) {
  const int m = 2 * h->n_cyc;
  CHECK(ensure_dq(h));
  h->cyc_raw = true;
  h->need_r = false;
  for (int j = 0; j < m; ++j) {
    HIPCALL(hipMemsetAsync(h->tmp, 0, sizeof(double) * h->n_col, h->stream));
    HIPCALL(hipMemsetAsync(h->x, 0, sizeof(double) * h->n_col, h->stream));
    hipLaunchKernelGGL(k_cyc_unit, dim3(1), dim3(1), 0, h->stream, h->tmp, h->d_cyc_rows, j);
    const int rc = launch_direct(h, 0.0, 1);
    if (rc != NX_OK) {
      h->cyc_raw = false;
      return rc;
    }
    h->seq += 1;
    CHECK(wait_published(h));
    HIPCALL(hipMemcpyAsync(h->cyc_z + (int64_t)j * h->n_col, h->x, sizeof(double) * h->n_col,
                           hipMemcpyDeviceToDevice, h->stream));
  }
  h->cyc_raw = false;
  hipLaunchKernelGGL(k_cyc_cap, dim3(1), dim3(256), 0, h->stream, csr_of(h), h->cyc_z, h->n_col,
                     h->d_cyc_rows, m, h->cyc_cap, h->cyc_cap + (int64_t)m * m);
  CHECK(cyc_invert(h));
  h->cyc_version = h->lhs_version;
  return NX_OK;
}

// Exact on this handle: one rank (no communicator, no group), the exact Schur-complement
// preconditioner (consistent mass) on a decomposition without grounded cycle chains.
// This rank can run the direct solve exactly: the exact Schur-complement preconditioner
// (consistent mass) on a decomposition without grounded cycle chains; with several ranks
// also the LDS sweeps (their mode kModeDirect) and the coarse step.
bool direct_local(const nx_network* h) {
  const bool multi = proc_rank(h) || h->group != nullptr || h->nranks > 1;
  // a graph with cycles: the Woodbury correction of its cycle chains (one rank, or every
  // rank's share of it: nx_set_cycles_team)
  const bool exact = h->tree_exact || (h->n_cyc > 0 && (!multi || h->cyc_team));
  // the LDS sweeps run it (their mode 3); the global-memory fallback (LDS caps exceeded)
  // leaves the solve to MINRES
  if (!(h->solver == 1 && h->pc && h->pc_lds && h->pa.exact && exact && h->E > 0)) return false;
  if (h->cond_mass) return false;  // an auxiliary handle (nx_set_cell_mass): not its own CSR
  // several ranks: the coarse step, and the residual formed by the down sweeps
  return !multi || (h->pc_jobs > 0 && h->pa.n_coarse > 0 && h->pa.n_coarse <= kCapCoarse &&
                    h->fres_ok);
}

// The ranks decide together: a group compares its handles here, RCCL ranks agreed in
// check_schedules (all-reduced with the schedule signature).
bool direct_applicable(const Team& t) {
  if (proc_rank(t.hs[0])) return t.hs[0]->sched_checked && t.hs[0]->direct_all;
  for (int r = 0; r < t.P; ++r)
    if (!direct_local(t.hs[r])) return false;
  return true;
}

// Several ranks (RCCL, one process per GPU; or an in-process group): every rank's fused
// sweeps in mode kModeDirect with the coarse all-reduce between the halves (every rank then
// solves the coarse forest redundantly -- same inputs, same order, same bits -- and
// back-substitutes from it), the halo of x (remote flux ends read by the multiplier rows),
// and one all-reduce of the residual sums, published by every rank.
// Several ranks: the cut rows ride in the residual's all-reduce (nx_set_cut given, fused
// check on, not disabled by NXHIP_DIR_CUT=0). Part of the schedule signature.
int build_left_cut(nx_network* h);
bool cut_mode(const nx_network* h);
// Several ranks, direct: k_pc_coarse's work in every down workgroup (pa.coarsedown; with the
// cut rows in the residual's all-reduce, whose reduce kernel then moves the top values into
// x). NXHIP_DIR_COARSE_DOWN=0 keeps the kernel. Part of the schedule signature.
bool coarse_down(const nx_network* h) {
  const char* e = std::getenv("NXHIP_DIR_COARSE_DOWN");
  const bool env = e == nullptr || std::atoi(e) != 0;
  return env && cut_mode(h) && h->pc_lds && h->pa.n_coarse > 0 && h->pc_jobs <= h->n_cu &&
         h->pa.n_coarse <= kCapCoarseLds && h->top_nt <= kTopThreads &&
         h->pa.n_top_lvl <= kMaxTopLvl;
}
bool cut_mode(const nx_network* h) {
  const char* e = std::getenv("NXHIP_DIR_CUT");  // read per solve: tests switch it
  const bool env = e == nullptr || std::atoi(e) != 0;
  return env && h->n_cut >= 0 && h->fres_ok && h->d_left_k != nullptr && h->cutbuf != nullptr;
}

// asmb (first pass): every rank's assembly is pending and heads its first half --
// k_dir_team_up where it applies (assembly + up sweep + top part in one launch), else the
// assembly kernel then the sweeps. check = false: the sweeps only (x = A^{-1} b, no residual
// and no publish -- the (k, 0) route's auxiliary solve, whose CSR is not its system).
int cyc_gather_team(const Team& t, bool prev);
int cyc_fix_team(const Team& t, double rtol, bool refine);
int launch_direct_team(const Team& t, double rtol, int refine, bool asmb = false,
                       bool check = true) {
  nx_network* h0 = t.hs[0];
  // graphs with cycles (nx_set_cycles_team): after the sweeps (A_g^{-1} b) the Woodbury
  // correction and the CSR's true residual publish; the sweeps' own residual is A_g's
  const bool cyc = h0->cyc_team && h0->n_cyc > 0 && !h0->cyc_raw;
  if (cyc && refine) CHECK(cyc_gather_team(t, true));  // U^T x before the correction's sweeps
  if (refine) {  // the previous pass's check left r = b - A x in tmp; its ghost slots 0
    for (int r = 0; r < t.P; ++r) {
      nx_network* h = t.hs[r];
      if (h->n_col > h->n_own)
        HIPCALL(hipMemsetAsync(h->tmp + h->n_own, 0, sizeof(double) * (h->n_col - h->n_own),
                               h->stream));
    }
  }
  for (int half = 0; half < 2; ++half) {
    for (int r = 0; r < t.P; ++r) {
      nx_network* h = t.hs[r];
      double* bin = refine ? h->tmp : h->rhs;
      h->pa.accum = refine ? 1 : 0;  // refinement: the sweeps add the correction to x
      h->pa.fres = h->fres_ok ? 1 : 0;  // and the down sweep the local rows' residual
      h->pa.coarsedown = coarse_down(h) ? 1 : 0;  // and the coarse step (no k_pc_coarse)
      if (half == 0 && asmb && !refine && dteam_on(h)) {
        launch_dteam(h);
      } else {
        if (half == 0 && asmb && !refine) CHECK(launch_assembly(h, 1, 1));
        launch_pc<true>(h, bin, bin, h->st, h->st + 1, kModeDirect, half, h->x);
      }
      h->pa.accum = 0;
      h->pa.fres = 0;
      h->pa.coarsedown = 0;
    }
    if (half == 0) CHECK(team_allreduce(t, -1, 3 * h0->pa.n_coarse));
  }
  if (!check) return NX_OK;
  if (cut_mode(h0)) {  // the cut rows ride in the residual's all-reduce: no halo of x
    for (int r = 0; r < t.P; ++r) {
      nx_network* h = t.hs[r];
      const int ntop = coarse_down(h) ? h->top_nt : 0;
      hipLaunchKernelGGL(k_dir_reduce_cut, dim3(1), dim3(kReduceThreads), 0, h->stream,
                         h->pa.rpart, h->pc_jobs, h->d_left, h->d_left_k, h->n_left, csr_of(h),
                         h->x, h->rhs, h->tmp, h->dir_bb, refine, h->n_cut, h->d_cut_own,
                         h->d_gk_off, h->d_gk_row, h->d_gk_coef, h->cutbuf,
                         h->pa.slot_lam + h->top_ts0, h->pa.slot_z + h->top_ts0, ntop);
    }
    CHECK(team_allreduce(t, -2, 2 + h0->n_cut));
    if (cyc) return cyc_fix_team(t, rtol, refine);
    for (int r = 0; r < t.P; ++r) {
      nx_network* h = t.hs[r];
      hipLaunchKernelGGL(k_dir_publish_cut, dim3(1), dim3(64), 0, h->stream, h->cutbuf,
                         h->n_cut, h->d_cut_own, h->tmp, rtol, h->d_seq, h->d_last);
    }
    HIPCALL(hipGetLastError());
    return NX_OK;
  }
  if (cyc) return cyc_fix_team(t, rtol, refine);
  CHECK(team_halo(t, VS_X, 0));
  for (int r = 0; r < t.P; ++r) {  // the down sweeps formed the local rows (direct_local:
    nx_network* h = t.hs[r];       // fres_ok); the rest need the halo of x
    hipLaunchKernelGGL(k_dir_reduce2_fr, dim3(1), dim3(kReduceThreads), 0, h->stream,
                       h->pa.rpart, h->pc_jobs, h->d_left, h->n_left, csr_of(h), h->x, h->rhs,
                       h->tmp, h->dir_bb, refine, h->red + 2);
  }
  CHECK(team_allreduce(t, 2, 2));
  for (int r = 0; r < t.P; ++r) {
    nx_network* h = t.hs[r];
    hipLaunchKernelGGL(k_dir_publish_red, dim3(1), dim3(64), 0, h->stream, h->red + 2, rtol,
                       h->d_seq, h->d_last);
  }
  HIPCALL(hipGetLastError());
  return NX_OK;
}

// ---- graphs with cycles, several ranks: the Woodbury correction across the ranks ---------
// U^T x over the ranks into cyc_u (prev: kept in cyc_prev, before a refinement pass's sweeps)
int cyc_gather_team(const Team& t, bool prev) {
  const int m = 2 * t.hs[0]->n_cyc;
  for (int r = 0; r < t.P; ++r) {
    nx_network* h = t.hs[r];
    hipLaunchKernelGGL(k_cyc_gather, dim3(1), dim3(256), 0, h->stream, h->x, h->d_cyc_rows, m,
                       h->cyc_u);
  }
  HIPCALL(hipGetLastError());
  CHECK(team_allreduce(t, -3, m));
  if (prev)
    for (int r = 0; r < t.P; ++r)
      HIPCALL(hipMemcpyAsync(t.hs[r]->cyc_prev, t.hs[r]->cyc_u, sizeof(double) * m,
                             hipMemcpyDeviceToDevice, t.hs[r]->stream));
  return NX_OK;
}

// After the sweeps: x -= Z Cinv U^T (x - x_before) on every rank's rows, then the true
// residual of A (the halo of x, every owned row from the CSR, the two sums over the ranks)
// published -- r kept in tmp for a refinement pass.
int cyc_fix_team(const Team& t, double rtol, bool refine) {
  const int m = 2 * t.hs[0]->n_cyc;
  CHECK(cyc_gather_team(t, false));
  for (int r = 0; r < t.P; ++r) {
    nx_network* h = t.hs[r];
    hipLaunchKernelGGL(k_cyc_w_team, dim3(grid_of(m, 256)), dim3(256), sizeof(double) * m, h->stream, h->cyc_u, m, h->cyc_cinv,
                       refine ? h->cyc_prev : nullptr, h->cyc_w);
    hipLaunchKernelGGL(k_cyc_fix, dim3(grid_of(h->n_own, kBlock)), dim3(kBlock), 0, h->stream,
                       h->x, h->cyc_z, h->n_col, h->cyc_w, m, h->n_own);
  }
  HIPCALL(hipGetLastError());
  CHECK(team_halo(t, VS_X, 0));
  for (int r = 0; r < t.P; ++r) {
    nx_network* h = t.hs[r];
    const int nrb = grid_of(h->n_own, kRowsPerBlock * res_chunks(h->n_own));
    hipLaunchKernelGGL(k_residual_ck, dim3(nrb), dim3(kBlock), 0, h->stream, csr_of(h), h->x,
                       h->rhs, h->partials, nrb, h->tmp, res_chunks(h->n_own));
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kReduceThreads), 0, h->stream, h->partials, nrb,
                       h->red + 2);
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kReduceThreads), 0, h->stream, h->partials + nrb,
                       nrb, h->red + 3);
  }
  HIPCALL(hipGetLastError());
  CHECK(team_allreduce(t, 2, 2));
  for (int r = 0; r < t.P; ++r) {
    nx_network* h = t.hs[r];
    hipLaunchKernelGGL(k_dir_publish_red, dim3(1), dim3(64), 0, h->stream, h->red + 2, rtol,
                       h->d_seq, h->d_last);
  }
  HIPCALL(hipGetLastError());
  return NX_OK;
}

// Z = A_g^{-1} U over the ranks (2K team tree solves of a unit right-hand side set by the
// row's owner, accumulated into zeroed x -- a refinement pass's shape), then every rank's
// share of U^T Z and of the couplings, summed over the ranks, and the same Cinv on every
// rank. Once per assembled matrix.
int cyc_build_team(const Team& t) {
  const int m = 2 * t.hs[0]->n_cyc;
  for (int r = 0; r < t.P; ++r) {
    CHECK(ensure_dq(t.hs[r]));
    t.hs[r]->cyc_raw = true;
  }
  int rc = NX_OK;
  for (int j = 0; j < m && rc == NX_OK; ++j) {
    for (int r = 0; r < t.P; ++r) {
      nx_network* h = t.hs[r];
      HIPCALL(hipMemsetAsync(h->tmp, 0, sizeof(double) * h->n_col, h->stream));
      HIPCALL(hipMemsetAsync(h->x, 0, sizeof(double) * h->n_col, h->stream));
      hipLaunchKernelGGL(k_cyc_unit, dim3(1), dim3(1), 0, h->stream, h->tmp, h->d_cyc_rows, j);
    }
    rc = launch_direct_team(t, 0.0, 1, false);
    for (int r = 0; r < t.P && rc == NX_OK; ++r) {
      nx_network* h = t.hs[r];
      h->seq += 1;
      rc = wait_published(h);
      if (rc == NX_OK && hipMemcpyAsync(h->cyc_z + (int64_t)j * h->n_col, h->x,
                                        sizeof(double) * h->n_col, hipMemcpyDeviceToDevice,
                                        h->stream) != hipSuccess)
        rc = fail(NX_ERR_HIP, "cycle correction: copying a column of Z failed");
    }
  }
  for (int r = 0; r < t.P; ++r) t.hs[r]->cyc_raw = false;
  CHECK(rc);
  for (int r = 0; r < t.P; ++r) {
    nx_network* h = t.hs[r];
    hipLaunchKernelGGL(k_cyc_cap_team, dim3(1), dim3(256), 0, h->stream, csr_of(h), h->cyc_z,
                       h->n_col, h->d_cyc_rows, m, h->d_cyc_qloc, h->d_cyc_lcol, h->cyc_cap,
                       h->cyc_cap + (int64_t)m * m);
  }
  HIPCALL(hipGetLastError());
  CHECK(team_allreduce(t, -4, m * m + m / 2));
  for (int r = 0; r < t.P; ++r) {
    CHECK(cyc_invert(t.hs[r]));
    t.hs[r]->cyc_version = t.hs[r]->lhs_version;
  }
  return NX_OK;
}

// The direct solve of a team (one rank, a group or an RCCL rank): one graph -- on one rank
// headed by the deferred assembly -- then the published true residual. The tree formula is
// exact but not backward stable to the last digits (its true residual is ~1e-13 .. 1e-11
// where a sparse LU reaches ~1e-15; the forward error stays ~1e-12): when the residual misses
// rtol, a second graph applies one step of iterative refinement (residual -> direct solve
// -> x += correction; ~1e-15 after it). Returns NX_OK with *converged = 0 if that is still
// above rtol (the caller runs MINRES). RCCL that refuses the capture: eager launches.
// One rank: the direct solve's five kernels are launched directly by default -- from an
// idle stream the first starts ~3 us after the call and the host enqueues the rest while
// it runs, where a graph replay costs ~10 us of fixed host time (C3: 0.0708 vs 0.0739
// ms/step, r02n A/B). Several ranks: graphs.
// (Measured and kept out: the down sweep's last workgroup publishing through an atomic
// ticket instead of k_dir_publish_fr -- 0.079 vs 0.072 ms/step: every workgroup's release
// fence writes back its XCD's L2, dirty with x, before the ticket.)

// ---- several ranks: the fused step with the device-side exchange (k_dir_xr / k_dir_xg) --
// slot strides: the exchange's doubles, then the writer's tag
constexpr int kXld1 = 3 * kCapCoarseLds + 1, kXld2 = 2 + kCapCoarseLds + 1;
size_t xmb_bytes(int P) {  // slots, 2P flags, P 64-bit abort words
  return sizeof(double) * (size_t)P * (kXld1 + kXld2) + sizeof(unsigned) * 4 * (size_t)P;
}
XPeer xpeer_of(void* base, int P) {
  XPeer x;
  x.mb1 = static_cast<double*>(base);
  x.mb2 = x.mb1 + (size_t)P * kXld1;
  x.fl = reinterpret_cast<unsigned*>(x.mb2 + (size_t)P * kXld2);
  return x;
}
// this rank's mailbox: fine-grained (uncached) device memory -- the peers write into it over
// xGMI and its reads must not hit a stale L2 line -- zeroed (flags start below every tag)
int xr_alloc(nx_network* h, int P) {
  if (h->xmb) return NX_OK;
  HIPCALL(hipExtMallocWithFlags(&h->xmb, xmb_bytes(P), hipDeviceMallocUncached));
  HIPCALL(hipMemset(h->xmb, 0, xmb_bytes(P)));
  HIPCALL(hipMalloc((void**)&h->d_xpeers, sizeof(XPeer) * P));
  return NX_OK;
}
void xr_free(nx_network* h) {
  for (void* q : h->xr_opened) (void)hipIpcCloseMemHandle(q);
  h->xr_opened.clear();
  if (h->xmb) (void)hipFree(h->xmb);
  if (h->d_xpeers) (void)hipFree(h->d_xpeers);
  h->xmb = nullptr;
  h->d_xpeers = nullptr;
  h->xr_linked = false;
}
int xr_link(nx_network* h, const std::vector<XPeer>& peers) {
  HIPCALL(hipMemcpy(h->d_xpeers, peers.data(), sizeof(XPeer) * peers.size(), hipMemcpyHostToDevice));
  h->xpeers_host = peers;  // (xr_settle posts an abort word from the host through them)
  h->xr_linked = true;
  h->sched_checked = false;  // (the ranks agree on the exchange in check_schedules)
  return NX_OK;
}
bool xr_variant(int v) { return v == 5 || v == 10 || v == 7 || v == 2; }  // <8,2|3|4>, <16,4>
size_t xr_static_lds(int v);  // the exchange kernels' static LDS (below)

// one rank's share of the decision: its tables, its peers linked, the coarse / cut sizes
// within the exchange's caps, one round of workgroups, the LDS
bool xr_local(const nx_network* h) {
  return h->xr_ok && h->xr_linked && h->pc && h->pc_lds && h->fres_ok && h->pa.exact &&
         h->n_cyc == 0 &&
         h->pc_jobs > 0 && h->pc_jobs <= h->n_cu && h->pa.n_coarse > 0 &&
         h->pa.n_coarse <= kCapCoarseLds && h->n_cut >= 0 && h->n_cut <= kCapCoarseLds &&
         h->top_nt > 0 && h->top_nt <= kTopThreads && h->pa.n_top_lvl <= kMaxTopLvl &&
         xr_variant(h->dstep_variant) &&
         h->dstep_lds + xr_static_lds(h->dstep_variant) <= 160 * 1024;
}
bool xr_env() {
  const char* e = std::getenv("NXHIP_DIR_XR");  // read per solve: tests switch it
  return e == nullptr || std::atoi(e) != 0;
}
// every rank runs it (group: all handles, co-resident in one launch; RCCL: check_schedules'
// agreement), the assembly pending everywhere (it heads the launch)
bool xr_on(const Team& t, bool with_asm) {
  if (!with_asm || !xr_env() || !team_multi(t)) return false;
  if (t.g) {
    int jobs = 0;
    for (int r = 0; r < t.P; ++r) {
      if (!xr_local(t.hs[r]) || t.hs[r]->dstep_variant != t.hs[0]->dstep_variant) return false;
      jobs += t.hs[r]->pc_jobs;
    }
    return jobs <= t.hs[0]->n_cu;
  }
  return t.hs[0]->sched_checked && t.hs[0]->xr_all && xr_local(t.hs[0]);
}

// The one-launch steps (k_dir_step, k_dir_xr, k_dir_xg) do not write the lumped flux mass
// dq: only the separate sweeps (a refinement pass, MINRES, the graph path) read it, and
// ensure_dq forms it before them. (4.2 MB of the step's stores at C3.)
// A job with more chains than one pass re-reads its chains' b and dq in phase 2: its step
// writes them (dstep_multi).
// NXHIP_DIR_SUP (read per launch: tests switch it): 0 off (phase 2 after the top values, as
// before round 6), 1 on (default), 3 on with the waiting workgroups' part after their stores
int dir_sup_mode() {
  const char* e = std::getenv("NXHIP_DIR_SUP");
  return e ? std::atoi(e) : 1;
}
// the superposition's instantiation runs this launch: asked for (and the park fits) and
// compiled for this lane shape
template <int CPL>
bool sup_launch(const DirStep& da) {
  return CPL <= 2 && (da.sup & 1) != 0;
}

DirStep dir_args(nx_network* h, double rtol) {
  h->dq_stale = !h->dstep_multi;
  DirStep d{h->edge_x, h->edge_R, h->edge_bc, h->edge_f, h->f, h->edge_lm, h->edge_seg,
                 h->val, h->rhs, h->dstep_multi ? h->dq : nullptr, h->nnz_lm, h->B, h->lm_val, h->val + h->nnz_edges,
                 h->rhs + h->n_edge_dofs, h->x, h->d_chain_post, h->d_left_off, h->n_left,
                 h->d_post, h->d_dsync, h->dstep_epoch, h->dstep_polls, rtol, h->seq + 1,
                 h->d_seq, h->d_last, h->dir_bb, h->d_job_hdr, h->d_crec, h->d_ci,
                 h->dstep_main, h->dstep_top, nullptr, XPeer{}, 0, 0, 0, 0, 0, 0u,
                 {kDirWaitPolls, kDirWaitPolls}, 0};
#ifdef NX_PHASE_TIMING
  if (const char* e = std::getenv("NXHIP_LEDGER")) d.ledger = std::atoi(e);
#endif
  d.sup = h->dstep_park && !h->dstep_multi ? dir_sup_mode() : 0;
  // (bit 2, the LDS copies: only asked for, and only when they fit -- measured neutral at
  // C3, r06l-r06o: the top solver is not the last workgroup of phase 2 any more)
  if (!h->dstep_rec) d.sup &= ~4;
  return d;
}
// the exchange fields of rank h's launch among X ranks (its own mailbox, the peers' table)
void xr_fill(nx_network* h, DirStep& da, int X) {
  da.n_left = h->xr_nleft;
  da.xpeers = h->d_xpeers;
  da.xself = xpeer_of(h->xmb, X);
  da.xP = X;
  da.xrank = h->rank;
  da.xld1 = kXld1;
  da.xld2 = kXld2;
  da.xK = h->n_cut;
  da.xtag = h->xtag;
  da.xpoll[0] = h->xpoll[0];
  da.xpoll[1] = h->xpoll[1];
}
// the dynamic LDS above 64 KiB, opted in once per kernel (not per launch)
void opt_in_lds(const void* fn, int bytes) {
  static thread_local std::vector<const void*> opted;
  if (std::find(opted.begin(), opted.end(), fn) != opted.end()) return;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  (void)hipGetLastError();
  opted.push_back(fn);
}

template <int W, int CPL>
int launch_xr_wc(const Team& t, double rtol) {
  // P: the handles launched here (a group's ranks, or this process's one rank);
  // X: the ranks exchanging (every rank of the group or of the communicator)
  const int P = t.P, X = t.g ? t.P : t.hs[0]->nranks;
  std::vector<DirStep> das(P);
  std::vector<int> goff(P + 1, 0);
  size_t lds = 0;
  for (int r = 0; r < P; ++r) {
    nx_network* h = t.hs[r];
    if (h->nranks != X) return fail(NX_ERR_STATE, "exchange step: rank count mismatch");
    h->xtag += 1;  // (the same on every rank: they launch together)
    DirStep da = dir_args(h, rtol);
    xr_fill(h, da, X);
    das[r] = da;
    goff[r + 1] = goff[r] + h->pc_jobs;
    lds = std::max(lds, h->dstep_lds);
  }
  if (t.g) {  // one launch of every rank's workgroups
    nx_group* g = t.g;
    const size_t bp = sizeof(PcArgs) * P, bd = sizeof(DirStep) * P, bo = sizeof(int) * (P + 1);
    if (!g->xg_dev) {
      HIPCALL(hipMalloc(&g->xg_dev, bp + bd + bo));
      HIPCALL(hipHostMalloc(&g->xg_host, bp + bd + bo, hipHostMallocDefault));
    }
    char* hb = static_cast<char*>(g->xg_host);
    for (int r = 0; r < P; ++r) std::memcpy(hb + sizeof(PcArgs) * r, &t.hs[r]->pa, sizeof(PcArgs));
    std::memcpy(hb + bp, das.data(), bd);
    std::memcpy(hb + bp + bd, goff.data(), bo);
    HIPCALL(hipMemcpyAsync(g->xg_dev, g->xg_host, bp + bd + bo, hipMemcpyHostToDevice, g->stream));
    const char* db = static_cast<const char*>(g->xg_dev);
    const int cap = (int)(160 * 1024 - xr_static_lds(t.hs[0]->dstep_variant));
    for (int r = 0; r < P; ++r) t.hs[r]->last_sup = sup_launch<CPL>(das[0]);
    if (sup_launch<CPL>(das[0])) {
      opt_in_lds(reinterpret_cast<const void*>(&k_dir_xg<W, CPL, CPL <= 2>), cap);
      hipLaunchKernelGGL((k_dir_xg<W, CPL, CPL <= 2>), dim3(goff[P]), dim3(kPcThreads), lds,
                         g->stream, reinterpret_cast<const PcArgs*>(db),
                         reinterpret_cast<const DirStep*>(db + bp),
                         reinterpret_cast<const int*>(db + bp + bd), P);
    } else {
      opt_in_lds(reinterpret_cast<const void*>(&k_dir_xg<W, CPL>), cap);
      hipLaunchKernelGGL((k_dir_xg<W, CPL>), dim3(goff[P]), dim3(kPcThreads), lds, g->stream,
                         reinterpret_cast<const PcArgs*>(db),
                         reinterpret_cast<const DirStep*>(db + bp),
                         reinterpret_cast<const int*>(db + bp + bd), P);
    }
    HIPCALL(hipStreamSynchronize(g->stream));  // (the pinned staging is rewritten next launch)
  } else {
    nx_network* h = t.hs[0];
    const int cap = (int)(160 * 1024 - xr_static_lds(h->dstep_variant));
    const bool prof = h->prof && h->dev[0];  // (events bound to the dispatch: bench.py)
    h->last_sup = sup_launch<CPL>(das[0]);
    if (sup_launch<CPL>(das[0])) {
      opt_in_lds(reinterpret_cast<const void*>(&k_dir_xr<W, CPL, CPL <= 2>), cap);
      hipExtLaunchKernelGGL((k_dir_xr<W, CPL, CPL <= 2>), dim3(h->pc_jobs), dim3(kPcThreads),
                            h->dstep_lds, h->stream, prof ? h->dev[0] : nullptr,
                            prof ? h->dev[1] : nullptr, 0, h->pa, das[0]);
    } else {
      opt_in_lds(reinterpret_cast<const void*>(&k_dir_xr<W, CPL>), cap);
      hipExtLaunchKernelGGL((k_dir_xr<W, CPL>), dim3(h->pc_jobs), dim3(kPcThreads),
                            h->dstep_lds, h->stream, prof ? h->dev[0] : nullptr,
                            prof ? h->dev[1] : nullptr, 0, h->pa, das[0]);
    }
  }
  HIPCALL(hipGetLastError());
  for (int r = 0; r < P; ++r) {
    t.hs[r]->dstep_epoch += 1;
    t.hs[r]->seq += 1;
  }
  return NX_OK;
}
int launch_xr(const Team& t, double rtol) {
  switch (t.hs[0]->dstep_variant) {
    case 5: return launch_xr_wc<8, 2>(t, rtol);
    case 10: return launch_xr_wc<8, 3>(t, rtol);
    case 7: return launch_xr_wc<8, 4>(t, rtol);
    default: return launch_xr_wc<16, 4>(t, rtol);
  }
}
size_t xr_static_lds(int v) {
  static size_t s[4] = {0, 0, 0, 0};
  const int i = v == 5 ? 0 : v == 7 ? 1 : v == 10 ? 3 : 2;
  if (!s[i]) {
    hipFuncAttributes a{};
    const void* fn = i == 0 ? reinterpret_cast<const void*>(&k_dir_xr<8, 2>)
                   : i == 1 ? reinterpret_cast<const void*>(&k_dir_xr<8, 4>)
                   : i == 3 ? reinterpret_cast<const void*>(&k_dir_xr<8, 3>)
                            : reinterpret_cast<const void*>(&k_dir_xr<16, 4>);
    s[i] = hipFuncGetAttributes(&a, fn) == hipSuccess ? a.sharedSizeBytes : 64 * 1024;
    if (i == 0) {  // (and the superposition's instantiation, the larger of the two)
      hipFuncAttributes b{};
      const size_t sb = hipFuncGetAttributes(&b, reinterpret_cast<const void*>(&k_dir_xr<8, 2, true>))
                                == hipSuccess ? b.sharedSizeBytes : 64 * 1024;
      s[i] = std::max(s[i], sb);
    }
  }
  return s[i];
}

// ---- after an exchange step: finished, or the ranks agree what to do ---------------------
// Whether rank h's launch published (finished), and if not why (sync[5]); then the hand-off
// counters and the host's count of published states are put back in step with the device.
int xr_settle(nx_network* h, bool* published) {
  const int rc = wait_published(h);
  *published = rc == NX_OK;
  if (rc == NX_OK) {
    h->xr_why = 0;
    return NX_OK;
  }
  if (rc != NX_ERR_STATE) return rc;
  (void)hipGetLastError();
  HIPCALL(hipStreamSynchronize(h->stream));
  unsigned sy[8];
  HIPCALL(hipMemcpy(sy, h->d_dsync, sizeof(sy), hipMemcpyDeviceToHost));
  h->xr_why = sy[5] ? sy[5] : (kXrFail1 | kXrFailLocal);
  if (!sy[5] && (int)h->xpeers_host.size() == h->nranks) {
    // no workgroup recorded a reason, so none wrote this launch's abort word either (the
    // advisor's r05 finding): post it from here, or a peer past exchange 1 would wait out
    // xr_host_finish's bound for this rank's exchange-2 share
    const unsigned long long w = ((unsigned long long)h->xr_why << 32) | h->xtag;
    for (int q = 0; q < h->nranks; ++q)
      if (q != h->rank)
        HIPCALL(hipMemcpy(reinterpret_cast<unsigned long long*>(h->xpeers_host[q].fl +
                                                                2 * h->nranks) + h->rank,
                          &w, sizeof(w), hipMemcpyHostToDevice));
  }
  HIPCALL(hipMemset(h->d_dsync, 0, 8 * sizeof(unsigned)));
  HIPCALL(hipMemcpy(&h->seq, h->d_seq, sizeof(int), hipMemcpyDeviceToHost));
  h->dstep_epoch = 0;
  return NX_OK;
}

bool xr_x_final(const nx_network* h) {
  return (h->xr_why & kXrFail2) && !(h->xr_why & kXrFail1);
}

// A rank whose launch gave up exchange 2 after passing exchange 1 holds its final x; only the
// residual's sum is missing. Whether the step can still finish is fixed by then: if every
// rank passed exchange 1, every rank wrote its exchange-2 slot and flag into every mailbox
// before it polled (so they arrive); if one did not, that rank never writes them and its
// abort word says so (reasons with kXrFail1, this launch's tag). So the host waits on its own
// mailbox for one or the other, and in the first case forms the sums and the residual
// exactly as dir_publish_xr does (rank order, no contraction: the same bits every other rank
// published) and takes the step as finished. Then every rank finishes a step, or none does.
constexpr double kXrHostWaitS = 60.0;
#pragma clang fp contract(off)
int xr_host_finish(nx_network* h, double rtol, bool* done) {
  const int X = h->nranks;
  const unsigned t = h->xtag;
  const XPeer me = xpeer_of(h->xmb, X);
  std::vector<unsigned> fl(4 * (size_t)X);
  std::vector<double> mb((size_t)X * kXld2);
  *done = false;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    HIPCALL(hipMemcpy(fl.data(), me.fl, sizeof(unsigned) * fl.size(), hipMemcpyDeviceToHost));
    const auto* ab = reinterpret_cast<const unsigned long long*>(fl.data() + 2 * X);
    bool all = true;
    for (int q = 0; q < X; ++q) {
      if ((unsigned)ab[q] == t && ((ab[q] >> 32) & kXrFail1)) return NX_OK;  // q stopped early
      all = all && fl[X + q] == t;
    }
    if (all) break;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kXrHostWaitS)
      return fail(NX_ERR_STATE, "exchange step: a rank's residual share never arrived");
    sched_yield();
  }
  HIPCALL(hipMemcpy(mb.data(), me.mb2, sizeof(double) * mb.size(), hipMemcpyDeviceToHost));
  const int K = h->n_cut, n = 2 + K;
  for (int q = 0; q < X; ++q)
    if (__builtin_bit_cast(unsigned long long, mb[(size_t)q * kXld2 + kXld2 - 1]) != t)
      return fail(NX_ERR_STATE, "exchange step: a residual slot holds another launch's data");
  std::vector<double> ys(n);
  for (int i = 0; i < n; ++i) {
    double v = 0.0;
    for (int q = 0; q < X; ++q) v += mb[(size_t)q * kXld2 + i];
    ys[i] = v;
  }
  double rr = ys[0];
  for (int k = 0; k < K; ++k) {
    const double rk = 0.0 - ys[2 + k];
    rr += rk * rk;
  }
  const double bb = ys[1];
  HIPCALL(hipMemcpy(h->dir_bb, &bb, sizeof(double), hipMemcpyHostToDevice));
  MrState* st = h->h_last;
  st->beta1 = std::sqrt(bb);
  st->relres = bb > 0.0 ? std::sqrt(rr / bb) : std::sqrt(rr);
  st->rtol = rtol;
  st->it = 1;
  st->done = 1;
  st->converged = st->relres <= rtol ? 1 : 0;
  *done = true;
  return NX_OK;
}
#pragma clang fp contract(on)

// The ranks of separate processes (RCCL, or the host transport) after a launch that no rank
// finished: one max-all-reduce of [tag, -tag] checks they are all at the same step -- by
// the construction above they are -- and every rank leaves the exchange step for good; the
// graph path solves this step. (A mismatch would pair collectives of different steps: it
// stops loudly instead.)
int xr_allmax(nx_network* h, double* v, int n) {
  if (!h->d_agree) CHECK(dalloc(&h->d_agree, 8));
  HIPCALL(hipMemcpy(h->d_agree, v, sizeof(double) * n, hipMemcpyHostToDevice));
  if (h->hcomm) {
    CHECK(hc_allreduce(h, h->d_agree, n, 1));
  } else {
    NCCLCALL(ncclAllReduce(h->d_agree, h->d_agree, n, ncclDouble, ncclMax, h->comm, h->stream));
    HIPCALL(hipStreamSynchronize(h->stream));
  }
  HIPCALL(hipMemcpy(v, h->d_agree, sizeof(double) * n, hipMemcpyDeviceToHost));
  return NX_OK;
}
int xr_agree(nx_network* h) {
  double v[2] = {(double)h->xtag, -(double)h->xtag};
  CHECK(xr_allmax(h, v, 2));
  h->xr_agreed += 1;
  h->xr_off = true;
  if (v[0] != -v[1]) return fail(NX_ERR_STATE, "exchange step: the ranks gave up different steps");
  return NX_OK;
}

enum XrOutcome { kXrDone = 0, kXrGraph = 1 };
// The exchange step of every rank of the team, settled: kXrDone (every rank holds its x and
// the same published residual, converged) or kXrGraph (the caller solves this step on the
// graph path: above rtol everywhere -- the assembly is done -- or given up everywhere, the
// exchange step then off for good and the assembly pending again).
int xr_conclude(nx_network* const* hs, int P, bool local, double rtol, int* outcome) {
  int fin = 0;
  for (int r = 0; r < P; ++r) {
    nx_network* h = hs[r];
    bool done = false;
    CHECK(xr_settle(h, &done));
    if (!done && xr_x_final(h)) CHECK(xr_host_finish(h, rtol, &done));
    if (done) {
      h->pend_lhs = h->pend_rhs = 0;  // (x final: the launch's assembly is complete too)
      h->last_dir_path = 3;
      fin += 1;
    }
  }
  *outcome = kXrGraph;
  if (fin == 0) {  // nobody finished: every rank leaves the exchange step here
    if (local) {
      for (int r = 0; r < P; ++r) {
        hs[r]->xr_off = true;
        hs[r]->xr_agreed += 1;
      }
    } else {
      CHECK(xr_agree(hs[0]));
    }
    return NX_OK;
  }
  if (fin != P) return fail(NX_ERR_STATE, "exchange step: some ranks finished the step, some not");
  const MrState s = *hs[0]->h_last;
  for (int r = 1; r < P; ++r)
    if (hs[r]->h_last->relres != s.relres && s.relres == s.relres)
      return fail(NX_ERR_STATE, "ranks disagree on the exchange step's residual");
  if (s.converged || s.relres != s.relres) *outcome = kXrDone;
  return NX_OK;
}
int run_xr(const Team& t, double rtol, int* outcome) {
  CHECK(launch_xr(t, rtol));
  return xr_conclude(t.hs, t.P, t.g != nullptr, rtol, outcome);
}

int solve_direct(const Team& t, double rtol, int32_t* iters, double* relres,
                 int32_t* converged) {
  const bool multi = team_multi(t);
  nx_network* h = t.hs[0];
  LeanGraphs& lg = lean_of(t);
  const bool prof1 = !multi && h->prof;  // events bound to the dispatches (profiling)
  if (prof1 && !h->dev[0])
    for (auto& e : h->dev) HIPCALL(hipEventCreate(&e));
  if (!multi && h->n_cyc > 0) {  // cycles: the correction of this matrix first
    CHECK(flush_assembly(h));
    if (h->cyc_version != h->lhs_version) CHECK(cyc_build(h));
  } else if (multi && h->cyc_team && h->n_cyc > 0) {  // (several ranks: built together)
    bool stale = false;
    for (int r = 0; r < t.P; ++r) {
      CHECK(flush_assembly(t.hs[r]));
      stale = stale || t.hs[r]->cyc_version != t.hs[r]->lhs_version;
    }
    if (stale) CHECK(cyc_build_team(t));
  }
  // the deferred assembly heads the solve (every rank's, several ranks)
  bool with_asm = true;
  for (int r = 0; r < t.P; ++r) with_asm = with_asm && t.hs[r]->pend_lhs && t.hs[r]->pend_rhs;
  for (int r = 0; r < t.P; ++r) t.hs[r]->last_dir_path = 0;
  if (multi && !h->xr_off && xr_on(t, with_asm)) {  // several ranks: one launch each
    if (!t.g && h->prof && !h->dev[0])
      for (auto& e : h->dev) HIPCALL(hipEventCreate(&e));
    int outcome = kXrGraph;
    CHECK(run_xr(t, rtol, &outcome));
    if (outcome == kXrDone) {
      if (!t.g && h->prof) {  // k_dir_xr's time (bench.py's roofline: one RCCL rank)
        HIPCALL(hipEventSynchronize(h->dev[1]));
        float ms = 0.f;
        HIPCALL(hipEventElapsedTime(&ms, h->dev[0], h->dev[1]));
        h->dir_ms[0] += ms;
        h->dir_cnt += 1;
      }
      const MrState s = *h->h_last;
      if (iters) *iters = 1;
      if (relres) *relres = s.relres;
      if (converged) *converged = s.converged;
      return NX_OK;
    }
    // the graph path solves this step again (run_xr cleared the pending assembly of the
    // ranks that finished it above rtol; a launch that gave up leaves it pending)
    with_asm = true;
    for (int r = 0; r < t.P; ++r) with_asm = with_asm && t.hs[r]->pend_lhs && t.hs[r]->pend_rhs;
  }
  if (with_asm && dstep_on(h)) {  // the fused step: assembly + solve + check in one launch
    const int rc = run_dstep(h, rtol, prof1);
    if (rc == NX_OK) {
      h->pend_lhs = h->pend_rhs = 0;
      h->last_dir_path = 1;
      if (prof1) {
        HIPCALL(hipEventSynchronize(h->dev[1]));
        float ms = 0.f;
        HIPCALL(hipEventElapsedTime(&ms, h->dev[0], h->dev[1]));
        h->dir_ms[0] += ms;
        h->dir_cnt += 1;
      }
      MrState s = *h->h_last;
      if (!s.converged && s.relres == s.relres) {  // one refinement step (forms r first)
        h->need_r = true;
        CHECK(ensure_dq(h));
        CHECK(launch_direct(h, rtol, 1));
        h->seq += 1;
        CHECK(wait_published(h));
        s = *h->h_last;
        s.it = 2;
      }
      if (iters) *iters = s.it;
      if (relres) *relres = s.relres;
      if (converged) *converged = s.converged;
      return NX_OK;
    }
    if (rc != NX_ERR_STATE) return rc;
    // a workgroup gave up waiting (they were not all resident): reset the hand-off counters
    // and take the four-launch path from now on (the assembly is still pending). The launch
    // published nothing, so the device's count of published states (d_seq, which the next
    // publish increments) is one behind the host's: take the host's back from the device,
    // or every later wait_published expects a stamp the publish kernels never write.
    (void)hipGetLastError();
    HIPCALL(hipStreamSynchronize(h->stream));
    HIPCALL(hipMemset(h->d_dsync, 0, 8 * sizeof(unsigned)));
    HIPCALL(hipMemcpy(&h->seq, h->d_seq, sizeof(int), hipMemcpyDeviceToHost));
    h->dstep_epoch = 0;
    h->dstep_off = true;
  }
  if (prof1) {  // eager, with events bound to the sweeps' and the residual's dispatches
    CHECK(flush_assembly(h));
    CHECK(ensure_dq(h));
    CHECK(launch_direct(h, rtol, 0, true));
    h->seq += 1;
    CHECK(wait_published(h));
    HIPCALL(hipStreamSynchronize(h->stream));
    const bool fused = h->pc_lds;
    for (int k = 0; k < 4; ++k) {
      if (k < 3 && !fused) continue;
      float ms = 0.f;
      if (k == 1 && fused && top_down_on(h))
        continue;  // no k_pc_top_lds dispatch (topdown): its events were not recorded
      if (hipEventElapsedTime(&ms, h->dev[2 * k], h->dev[2 * k + 1]) == hipSuccess)
        h->dir_ms[k] += ms;
      else
        (void)hipGetLastError();  // an event pair this solve did not record
    }
    h->dir_cnt += 1;
    const MrState s = *h->h_last;
    if (iters) *iters = s.it;
    if (relres) *relres = s.relres;
    if (converged) *converged = s.converged;
    return NX_OK;
  }
  for (int r = 0; r < t.P; ++r)
    if (!with_asm) {
      CHECK(flush_assembly(t.hs[r]));
      CHECK(ensure_dq(t.hs[r]));  // (the graphs below read it; an assembly heading them writes it)
    }
  // (measured and kept out: forking the CSR values' assembly onto a second graph branch
  // beside the sweeps -- the cross-queue dependencies cost ~13 us at the fork and ~9 us at
  // the join, more than the 17 us assembly they would hide; r02 trace)
  auto body = [&](int refine, bool asmb) -> int {
    if (multi) return launch_direct_team(t, rtol, refine, asmb);
    if (asmb) CHECK(launch_assembly(h, 1, 1));
    return launch_direct(h, rtol, refine);
  };
  // several ranks: graph replay; one rank: the launches issued directly
  const bool graphs = (!proc_rank(h) || h->rccl_graph_ok) && multi;
  auto run = [&](hipGraphExec_t* exec, hipGraph_t* graph, int* len, double* grtol, int key,
                 int refine, bool asmb) -> int {
    if (graphs && (!*exec || *grtol != rtol || *len != key)) {
      CHECK(drop_one(exec, graph, len));
      const int rc = capture(h, graph, exec, [&] { return body(refine, asmb); });
      if (rc != NX_OK && proc_rank(h)) {  // RCCL refused the capture: eager from now on
        (void)hipGetLastError();
        h->rccl_graph_ok = false;
      } else {
        CHECK(rc);
        *len = key;
        *grtol = rtol;
      }
    }
    h->last_graph = graphs && h->rccl_graph_ok;
    if (h->last_graph) {
      HIPCALL(hipGraphLaunch(*exec, h->stream));
    } else {
      CHECK(body(refine, asmb));
    }
    for (int r = 0; r < t.P; ++r) t.hs[r]->seq += 1;
    for (int r = 0; r < t.P; ++r) CHECK(wait_published(t.hs[r]));
    const MrState& s0 = *h->h_last;
    for (int r = 1; r < t.P; ++r)  // every rank published the same all-reduced sums
      if (t.hs[r]->h_last->relres != s0.relres && s0.relres == s0.relres)
        return fail(NX_ERR_STATE, "ranks disagree on the direct solve's residual");
    return NX_OK;
  };
  hipGraphExec_t* exec = with_asm ? &lg.direct_asm_exec : &lg.direct_exec;
  hipGraph_t* graph = with_asm ? &lg.direct_asm_graph : &lg.direct_graph;
  int* len = with_asm ? &lg.direct_asm_len : &lg.direct_len;
  double* grtol = with_asm ? &lg.direct_asm_rtol : &lg.direct_rtol;
  CHECK(run(exec, graph, len, grtol, 1, 0, with_asm));
  for (int r = 0; r < t.P; ++r) t.hs[r]->pend_lhs = t.hs[r]->pend_rhs = 0;
  MrState s = *h->h_last;
  if (!s.converged && s.relres == s.relres) {  // one refinement step (graph kept in lchunk;
                                                // MINRES continuation chunks use len > 0)
    CHECK(run(&lg.lchunk_exec, &lg.lchunk_graph, &lg.lchunk_len, &lg.lchunk_rtol, -1, 1, false));
    s = *h->h_last;
    s.it = 2;
  }
  if (iters) *iters = s.it;
  if (relres) *relres = s.relres;
  if (converged) *converged = s.converged;
  return NX_OK;
}

// 1: one graph per solve where possible (default; nx_set_lean(0): the
// general path with eager prologue and chunked iterations)
int& lean_flag() {  // nx_set_lean
  static int f = 1;
  return f;
}
bool lean_mode() { return lean_flag() != 0; }

// The lean solve of a team (single rank, group or RCCL rank). Returns NX_ERR_RCCL if the
// RCCL capture failed (the caller falls back to eager launches).
int solve_lean(const Team& t, double rtol, int32_t maxit, int L, int32_t* iters, double* relres,
               int32_t* converged) {
  const bool multi = team_multi(t);
  nx_network* h0 = t.hs[0];
  for (int r = 0; r < t.P; ++r) {  // the iterations use the factored coefficients
    nx_network* h = t.hs[r];
    h->pa.factored = h->pa.dc_kappa ? 1 : 0;
    h->pa.mdense = (multi && h->pa.dense && h->pa.KJ && h->pa.n_coarse > 0 && h->pa.lin) ? 1 : 0;
    // the down sweep of iteration k packs the halo of iteration k+1 (fused coarse solve and
    // point-to-point beta^2 only)
    h->pa.fuse_pack = (multi && h->pa.fused && h->pa.mdense && h->beta_p2p && h->pc_lds) ? 1 : 0;
    h->pa.send_idx = h->send_idx;
    h->pa.n_send = h->send_off.empty() ? 0 : h->send_off.back();
    h->pa.send_buf = h->send_buf;
    h->pa.red1 = h->red + 1;
    h->pa.gath_self = h->gath ? h->gath + h->rank : nullptr;
  }
  LeanGraphs& lg = lean_of(t);
  auto cap = [&](hipGraph_t* graph, hipGraphExec_t* exec, const std::function<int()>& body) {
    const int rc = capture(h0, graph, exec, body);
    if (rc != NX_OK && proc_rank(h0)) {  // RCCL refused the capture: eager from now on
      (void)hipGetLastError();
      h0->rccl_graph_ok = false;
      return (int)NX_ERR_RCCL;
    }
    return rc;
  };
  if (!lg.head_exec || lg.head_len != L || lg.head_rtol != rtol || lg.head_maxit != maxit) {
    CHECK(drop_one(&lg.head_exec, &lg.head_graph, &lg.head_len));
    CHECK(cap(&lg.head_graph, &lg.head_exec, [&] {
      return multi ? launch_head_multi(t, L, rtol, maxit) : launch_head_lean(h0, L, rtol, maxit);
    }));
    lg.head_len = L;
    lg.head_rtol = rtol;
    lg.head_maxit = maxit;
  }
  h0->last_graph = true;
  HIPCALL(hipGraphLaunch(lg.head_exec, h0->stream));
  for (int r = 0; r < t.P; ++r) t.hs[r]->seq += 1;
  for (;;) {
    // the graph's last k_mr_a published the state it ends with (the final one once done);
    // the solution update may still be running -- later work on the stream is ordered
    // after it and every host read of device data synchronises the stream
    for (int r = 0; r < t.P; ++r) CHECK(wait_published(t.hs[r]));
    const MrState& s0 = *h0->h_last;
    for (int r = 1; r < t.P; ++r) {  // the ranks run the same recurrence on the same scalars
      const MrState& o = *t.hs[r]->h_last;
      if (o.it != s0.it || o.done != s0.done || o.relres != s0.relres) {
        char msg[256];
        std::snprintf(msg, sizeof(msg), "ranks diverged: rank %d it %d done %d relres %.17g vs "
                      "rank 0 it %d done %d relres %.17g", r, o.it, o.done, o.relres, s0.it,
                      s0.done, s0.relres);
        return fail(NX_ERR_STATE, msg);
      }
    }
    if (s0.done) break;
    if (!lg.lchunk_exec || lg.lchunk_len != L) {
      CHECK(drop_one(&lg.lchunk_exec, &lg.lchunk_graph, &lg.lchunk_len));
      CHECK(cap(&lg.lchunk_graph, &lg.lchunk_exec, [&] {
        for (int k = L; k < 2 * L; ++k) {
          if (multi) {
            CHECK(launch_part_pc(t, k));
            const LeanOpt next{false, k + 1 == 2 * L, rtol, maxit};
            CHECK(launch_part_a(t, k + 1, &next));
          } else {
            CHECK(team_pc(t, k, 0));
            launch_a_lean(h0, k + 1, false, rtol, maxit, nullptr, k + 1 == 2 * L);
          }
        }
        HIPCALL(hipGetLastError());
        return NX_OK;
      }));
      lg.lchunk_len = L;
    }
    HIPCALL(hipGraphLaunch(lg.lchunk_exec, h0->stream));
    for (int r = 0; r < t.P; ++r) t.hs[r]->seq += 1;
  }
  const MrState s = *h0->h_last;
  if (iters) *iters = s.it;
  if (relres) *relres = s.relres;
  if (converged) *converged = s.converged;
  return NX_OK;
}

// MINRES of every rank of the team (nx_solve / nx_group_solve).
// What decides the exchange schedule of a multi-rank solve: every rank must run the same
// one (a rank on the global-memory preconditioner kernels while another runs the LDS
// kernels' linear form would pair different collectives). Each rank decides from its own
// decomposition (LDS caps), so the ranks compare.
constexpr int kSchedSig = 11;
bool direct_local(const nx_network* h);
bool cut_mode(const nx_network* h);
bool coarse_down(const nx_network* h);
void sched_sig(const nx_network* h, int* s) {
  s[0] = h->pc;
  s[1] = h->pc && h->pc_lds;
  s[2] = h->pc ? h->pa.lin : 0;
  s[3] = h->pc ? h->pa.fused : 0;
  s[4] = h->pc ? h->pc_variant : 0;
  s[5] = h->beta_p2p;
  // the dense top (nx_set_pc_dense, decided per rank from its kMaxNeed fit) drives mdense
  // and with it fuse_pack: who packs the halo and beta^2 -- a per-rank difference would
  // leave peers reading stale halo values
  s[6] = h->pc ? h->pa.dense : 0;
  s[7] = h->pc ? (h->pa.n_coarse > 0) : 0;
  // the direct solve's residual: halo of x + all-reduce of 2, or one all-reduce of 2 + K
  s[8] = cut_mode(h) ? 1 + h->n_cut : 0;
  s[9] = coarse_down(h) ? 1 : 0;  // the coarse step in the down sweeps or k_pc_coarse
  s[10] = h->n_cyc;  // the cycle correction's all-reduces (nx_set_cycles_team)
}

int check_schedules(const Team& t) {
  int s0[kSchedSig], s[kSchedSig];
  sched_sig(t.hs[0], s0);
  for (int r = 1; r < t.P; ++r) {
    sched_sig(t.hs[r], s);
    for (int i = 0; i < kSchedSig; ++i)
      if (s[i] != s0[i])
        return fail(NX_ERR_STATE, "ranks chose different kernel schedules (rank " +
                                      std::to_string(r) + ", item " + std::to_string(i) + ")");
  }
  nx_network* h = t.hs[0];
  if (!proc_rank(h) || h->sched_checked) return NX_OK;
  // max of s and of -s over the ranks: equal iff all ranks agree; the last entry is the
  // max of -direct_local: the direct solve runs only if every rank can run it
  int v[2 * kSchedSig + 2];
  for (int i = 0; i < kSchedSig; ++i) {
    v[i] = s0[i];
    v[kSchedSig + i] = -s0[i];
  }
  v[2 * kSchedSig] = direct_local(h) ? -1 : 0;
  v[2 * kSchedSig + 1] = xr_local(h) ? -1 : 0;  // the exchange step only if every rank can
  int* d = nullptr;
  HIPCALL(hipMalloc((void**)&d, sizeof(v)));
  int rc = NX_OK;
  if (hipMemcpy(d, v, sizeof(v), hipMemcpyHostToDevice) != hipSuccess ||
      (h->hcomm ? hc_allreduce(h, d, 2 * kSchedSig + 2, 1) != NX_OK
                : ncclAllReduce(d, d, 2 * kSchedSig + 2, ncclInt32, ncclMax, h->comm, h->stream) !=
                      ncclSuccess) ||
      hipStreamSynchronize(h->stream) != hipSuccess ||
      hipMemcpy(v, d, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(NX_ERR_RCCL, "kernel schedule comparison across ranks failed");
  (void)hipFree(d);
  if (rc != NX_OK) return rc;
  for (int i = 0; i < kSchedSig; ++i)
    if (v[i] != -v[kSchedSig + i])
      return fail(NX_ERR_STATE, "ranks chose different kernel schedules (item " +
                                    std::to_string(i) + ": preconditioner decomposition "
                                    "outside the LDS caps on some ranks)");
  h->direct_all = v[2 * kSchedSig] == -1;
  h->xr_all = v[2 * kSchedSig + 1] == -1;
  h->sched_checked = true;
  return NX_OK;
}

// (k, 0) through the condensed P1/DG0 system (nx_fe_set_direct): condense the right-hand
// side (and, first pass, the auxiliary lumped mass) on this handle's stream, the auxiliary
// handle's tree solve on its stream, expand, then this CSR's true residual, published. Up
// to two refinement passes (x += the same solve of r). *converged = 0 when still above
// rtol: the caller runs MINRES. Several ranks (process ranks: RCCL or the host transport):
// the auxiliary solve is the ranks' direct tree solve (launch_direct_team: the coarse step's
// all-reduce, the cut rows), condense and expand stay per edge, and the true residual takes
// the halo of x and one all-reduce of two sums.
void fe_true_residual(nx_network* h, double rtol, int nrb);
int fe_true_residual_team(nx_network* h, double rtol, int nrb) {
  nx_network* hs[1] = {h};
  const Team t{hs, 1, nullptr};
  CHECK(team_halo(t, VS_X, 0));
  hipLaunchKernelGGL(k_residual_ck, dim3(nrb), dim3(kBlock), 0, h->stream, csr_of(h), h->x,
                     h->rhs, h->partials, nrb, h->tmp, res_chunks(h->n_own));
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kReduceThreads), 0, h->stream, h->partials, nrb,
                     h->red + 2);
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kReduceThreads), 0, h->stream, h->partials + nrb,
                     nrb, h->red + 3);
  HIPCALL(hipGetLastError());
  CHECK(team_allreduce(t, 2, 2));
  hipLaunchKernelGGL(k_dir_publish_red, dim3(1), dim3(64), 0, h->stream, h->red + 2, rtol,
                     h->d_seq, h->d_last);
  HIPCALL(hipGetLastError());
  return NX_OK;
}
// The couplings a = A[q, lam] of the cycle chains' grounded ends from the P1 layout's rows
// (the auxiliary handle holds no assembled CSR): a flux end q is its edge's q_0 (-1 at the
// source multiplier) or q_N (+1 at the target's) -- k_pattern's entries; then U^T Z as
// k_cyc_cap forms it.
__global__ __launch_bounds__(256) void k_cyc_cap_p1(const double* __restrict__ Z, int64_t ldz,
                                                    const int* __restrict__ rows, int m, int N,
                                                    double* __restrict__ cap,
                                                    double* __restrict__ acoef) {
  for (int i = threadIdx.x; i < m * m; i += 256) {
    const int r = i / m, c = i % m;
    cap[i] = Z[(int64_t)c * ldz + rows[r]];
  }
  for (int k = threadIdx.x; 2 * k < m; k += 256) {
    const int loc = rows[2 * k] % (2 * N + 1);
    acoef[k] = loc == 0 ? -1.0 : (loc == 2 * N ? 1.0 : 0.0);  // (0: cyc_invert refuses it)
  }
}

// Several ranks: this rank's share of U^T Z (the rows of U it owns) and the couplings of the
// cycle chains it holds, by the flux end's position in the P1 layout (k_cyc_cap_team's, with
// no CSR values: the auxiliary handle holds none)
__global__ __launch_bounds__(256) void k_cyc_cap_team_p1(const double* __restrict__ Z, int64_t ldz,
                                                         const int* __restrict__ own, int m,
                                                         const int* __restrict__ qloc, int N,
                                                         double* __restrict__ cap,
                                                         double* __restrict__ acoef) {
  for (int i = threadIdx.x; i < m * m; i += 256) {
    const int r = i / m, c = i % m;
    cap[i] = own[r] >= 0 ? Z[(int64_t)c * ldz + own[r]] : 0.0;
  }
  for (int k = threadIdx.x; 2 * k < m; k += 256) {
    double a = 0.0;
    if (qloc[k] >= 0) {
      const int loc = qloc[k] % (2 * N + 1);
      a = loc == 0 ? -1.0 : (loc == 2 * N ? 1.0 : 0.0);
    }
    acoef[k] = a;  // (summed over the ranks: one rank holds each chain)
  }
}

// Several ranks: the auxiliary handle's team Woodbury correction (nx_set_cycles_team on it):
// Z by the ranks' tree solves of unit right-hand sides (sweeps only, the coarse all-reduce
// between their halves), U^T Z and the couplings summed over the ranks, Cinv on every rank
int fe_cyc_build_team(nx_network* h, nx_network* a) {
  const int m = 2 * a->n_cyc;
  const hipStream_t as = a->stream;
  a->stream = h->stream;
  a->need_r = false;
  a->cyc_raw = true;
  nx_network* ah[1] = {a};
  const Team t{ah, 1, nullptr};
  int rc = NX_OK;
  for (int j = 0; j < m && rc == NX_OK; ++j) {
    if (hipMemsetAsync(a->tmp, 0, sizeof(double) * a->n_col, a->stream) != hipSuccess ||
        hipMemsetAsync(a->x, 0, sizeof(double) * a->n_col, a->stream) != hipSuccess) {
      rc = fail(NX_ERR_HIP, "fe_cyc_build_team: memset");
      break;
    }
    hipLaunchKernelGGL(k_cyc_unit, dim3(1), dim3(1), 0, a->stream, a->tmp, a->d_cyc_rows, j);
    rc = launch_direct_team(t, 0.0, 1, false, false);
    if (rc == NX_OK &&
        hipMemcpyAsync(a->cyc_z + (int64_t)j * a->n_col, a->x, sizeof(double) * a->n_col,
                       hipMemcpyDeviceToDevice, a->stream) != hipSuccess)
      rc = fail(NX_ERR_HIP, "fe_cyc_build_team: copy");
  }
  a->cyc_raw = false;
  if (rc == NX_OK) {
    hipLaunchKernelGGL(k_cyc_cap_team_p1, dim3(1), dim3(256), 0, a->stream, a->cyc_z, a->n_col,
                       a->d_cyc_rows, m, a->d_cyc_qloc, (int)a->N, a->cyc_cap,
                       a->cyc_cap + (int64_t)m * m);
    rc = team_allreduce(t, -4, m * m + m / 2);
  }
  if (rc == NX_OK) rc = cyc_invert(a);
  a->stream = as;
  CHECK(rc);
  a->cyc_version = h->lhs_version;
  return NX_OK;
}

// (k, 0) on a graph with cycles (one rank): the auxiliary handle's Woodbury correction for
// the condensed system (nx_set_cycles on the auxiliary handle): Z = A_g^{-1} U by its tree
// solves of unit right-hand sides (the condensed lumped mass just written by k_fe_condense),
// U^T Z and the couplings, Cinv on the host. On this handle's stream; once per assembled
// matrix of h (its coefficients: the condensed mass is R h [[a, b], [b, a]]).
int fe_cyc_build(nx_network* h, nx_network* a) {
  const int m = 2 * a->n_cyc;
  const hipStream_t as = a->stream;
  a->stream = h->stream;
  a->need_r = false;
  int rc = NX_OK;
  for (int j = 0; j < m && rc == NX_OK; ++j) {
    if (hipMemsetAsync(a->tmp, 0, sizeof(double) * a->n_col, a->stream) != hipSuccess ||
        hipMemsetAsync(a->x, 0, sizeof(double) * a->n_col, a->stream) != hipSuccess) {
      rc = fail(NX_ERR_HIP, "fe_cyc_build: memset");
      break;
    }
    hipLaunchKernelGGL(k_cyc_unit, dim3(1), dim3(1), 0, a->stream, a->tmp, a->d_cyc_rows, j);
    rc = launch_direct(a, 0.0, 1);  // (refinement form: x += A_g^{-1} tmp; sweeps only)
    if (rc == NX_OK &&
        hipMemcpyAsync(a->cyc_z + (int64_t)j * a->n_col, a->x, sizeof(double) * a->n_col,
                       hipMemcpyDeviceToDevice, a->stream) != hipSuccess)
      rc = fail(NX_ERR_HIP, "fe_cyc_build: copy");
  }
  if (rc == NX_OK) {
    hipLaunchKernelGGL(k_cyc_cap_p1, dim3(1), dim3(256), 0, a->stream, a->cyc_z, a->n_col,
                       a->d_cyc_rows, m, (int)a->N, a->cyc_cap, a->cyc_cap + (int64_t)m * m);
    rc = cyc_invert(a);
  }
  a->stream = as;
  CHECK(rc);
  a->cyc_version = h->lhs_version;
  return NX_OK;
}

int fe_solve_direct(nx_network* h, double rtol, int32_t* iters, double* relres,
                    int32_t* converged) {
  nx_network* a = h->fe_aux;
  const bool ranks = proc_rank(h);
  CHECK(flush_assembly(h));
  const bool apend = a->pend_lhs || a->pend_rhs;
  CHECK(flush_assembly(a));
  if (apend) {  // (the auxiliary handle's own assembly ran on its stream)
    HIPCALL(hipEventRecord(h->fe_ev[1], a->stream));
    HIPCALL(hipStreamWaitEvent(h->stream, h->fe_ev[1], 0));
  }
  const FeCond c{h->edge_x, h->edge_R, h->N, h->fe_k - 1, h->E, h->fe_slot, h->fe_vfe,
                 h->fe_vaux, h->fe_ife, h->fe_pfe, h->fe_paux, h->fe_lfe, h->fe_laux, h->fe_nl,
                 h->fe_cst, h->fe_ab, h->fe_cellh};
  const int64_t nv = h->E * (h->N + 1), np = h->E * (int64_t)h->N, n0 = nv + np + h->fe_nl;
  const int nrb = grid_of(h->n_own, kRowsPerBlock * res_chunks(h->n_own));
  MrState s{};
  int pass = 0;
  h->last_dir_path = 2;  // the condensed route (nx_get_direct_path)
  for (; pass < 3; ++pass) {
    const double* b = pass ? h->tmp : h->rhs;  // refinement: the residual the check kept
    hipLaunchKernelGGL(k_fe_condense, dim3(grid_of(n0, kBlock)), dim3(kBlock), 0, h->stream, c,
                       b, pass ? nullptr : a->dq, a->rhs);
    // a graph with cycles: Woodbury (one rank; several: the team's, a->cyc_team)
    const int mcyc = (!ranks || a->cyc_team) ? 2 * a->n_cyc : 0;
    if (mcyc && pass == 0 && a->cyc_version != h->lhs_version)
      CHECK(ranks ? fe_cyc_build_team(h, a) : fe_cyc_build(h, a));
    {  // the auxiliary tree solve on this handle's stream (no cross-queue hand-offs)
      const hipStream_t as = a->stream;
      a->stream = h->stream;
      nx_network* ah[1] = {a};
      const int rc = ranks ? launch_direct_team(Team{ah, 1, nullptr}, 0.0, 0, false, false)
                           : launch_direct(a, 0.0, 0);
      a->stream = as;
      CHECK(rc);
    }
    if (mcyc && !ranks) {  // x_aux -= Z Cinv U^T x_aux: the couplings the tree solve dropped
      hipLaunchKernelGGL(k_cyc_w, dim3(grid_of(mcyc, 256)), dim3(256), sizeof(double) * mcyc, h->stream, a->x, a->d_cyc_rows, mcyc,
                         a->cyc_cinv, nullptr, a->cyc_w, nullptr);
      hipLaunchKernelGGL(k_cyc_fix, dim3(grid_of(a->n_own, kBlock)), dim3(kBlock), 0, h->stream,
                         a->x, a->cyc_z, a->n_col, a->cyc_w, mcyc, a->n_own);
    } else if (mcyc) {  // several ranks: U^T x_aux summed over them first
      const hipStream_t as = a->stream;
      a->stream = h->stream;
      nx_network* ah[1] = {a};
      const int rc = cyc_gather_team(Team{ah, 1, nullptr}, false);
      if (rc == NX_OK) {
        hipLaunchKernelGGL(k_cyc_w_team, dim3(grid_of(mcyc, 256)), dim3(256),
                           sizeof(double) * mcyc, h->stream, a->cyc_u, mcyc, a->cyc_cinv, nullptr,
                           a->cyc_w);
        hipLaunchKernelGGL(k_cyc_fix, dim3(grid_of(a->n_own, kBlock)), dim3(kBlock), 0,
                           h->stream, a->x, a->cyc_z, a->n_col, a->cyc_w, mcyc, a->n_own);
      }
      a->stream = as;
      CHECK(rc);
    }
    hipLaunchKernelGGL(k_fe_expand, dim3(grid_of(n0 + np, kBlock)), dim3(kBlock), 0, h->stream,
                       c, a->x, b, h->x, pass);
    if (ranks)
      CHECK(fe_true_residual_team(h, rtol, nrb));
    else
      fe_true_residual(h, rtol, nrb);
    HIPCALL(hipGetLastError());
    h->seq += 1;
    CHECK(wait_published(h));
    s = *h->h_last;
    if (s.converged || s.relres != s.relres) break;
  }
  if (iters) *iters = std::min(pass, 2) + 1;
  if (relres) *relres = s.relres;
  if (converged) *converged = s.converged;
  return NX_OK;
}

// Continuous pressure (k > m >= 1) on one rank, a forest (nx_fe_set_cp): the node-condensed
// direct solve -- per edge its forward sweep, the node forest level by level, per edge
// its back-substitution -- then this CSR's true residual, published. Up to two refinement
// passes (the same solve of r = b - A x, added). *converged = 0 when still above rtol: the
// caller runs MINRES.
// A general-degree handle's true residual r = b - A x (kept in tmp for a refinement pass) and
// its published relres: from the edge templates while the CSR holds the assembled
// coefficients (no CSR reads for the edges' rows), else from the CSR
void fe_true_residual(nx_network* h, double rtol, int nrb) {
  if (fe_tpl_on(h) && h->asm_coef_version == h->coef_version) {
    const int lb = grid_of(h->n_own - h->E * (int64_t)fe_per(h), 64 * kFesWaves);
    const int eb = std::max(1, std::min(fe_tpl_blocks(h), h->nblk - lb));
    const FeArgs fa{h->edge_x, h->edge_R, h->edge_bc, h->f, h->edge_f, h->N, h->fe_kind,
                    h->fe_tval, h->fe_aptr, h->fe_aidx, h->fe_aent, h->fe_bptr, h->fe_bidx,
                    h->fe_bent, h->nnz, h->n_own, h->val, h->rhs, 1, 0, h->E, h->fe_cellh};
    hipLaunchKernelGGL(k_fe_tres, dim3(eb + lb), dim3(64 * kFesWaves), fe_tpl_lds_of(h, true),
                       h->stream, fa, fe_tpl_args(h, eb), csr_of(h), h->x, h->rhs, h->tmp,
                       h->partials, eb + lb);
    hipLaunchKernelGGL(k_dir_publish, dim3(1), dim3(kReduceThreads), 0, h->stream, h->partials,
                       eb + lb, rtol, h->d_seq, h->d_last);
    return;
  }
  hipLaunchKernelGGL(k_residual_ck, dim3(nrb), dim3(kBlock), 0, h->stream, csr_of(h), h->x,
                     h->rhs, h->partials, nrb, h->tmp, res_chunks(h->n_own));
  hipLaunchKernelGGL(k_dir_publish, dim3(1), dim3(kReduceThreads), 0, h->stream, h->partials,
                     nrb, rtol, h->d_seq, h->d_last);
}

// NXHIP_CP_PIPE=0: the node forest's one-workgroup levels without the pipelining (A/B)
bool cp_pipe_on() {
  const char* e = std::getenv("NXHIP_CP_PIPE");
  return e == nullptr || std::atoi(e) != 0;
}

// The node forest's solve: levels of more than kCpWide nodes as grid launches (a thread per
// node), the runs of narrower levels in one workgroup each; up deepest first, then down.
void cp_nodes_launch(nx_network* h, const CpArgs& a, const CpTree& tr, const double* b) {
  const std::vector<int>& lo = h->cp_lev_host;
  const int nl = h->cp_nlev;
  // (pipelined: levels of more than 1024 nodes go to the grid launches)
  const int wmax = tr.rec != nullptr && cp_pipe_on() ? 1024 : kCpWide;
  auto wide = [&](int L) { return lo[L + 1] - lo[L] > wmax; };
  for (int up = 1; up >= 0; --up) {
    // runs of levels in the pass's order: a wide level alone, consecutive narrow ones together
    int k = 0;
    while (k < nl) {
      const int L = up ? nl - 1 - k : k;
      const nx_network::CpRun* run = nullptr;  // a run of wide levels in subtree chunks
      if (wmax == 1024)
        for (const auto& r : h->cp_runs)
          if (up ? L == r.L1 - 1 : L == r.L0) run = &r;
      if (run != nullptr) {
        hipLaunchKernelGGL(k_cp_nodes_rec, dim3(run->nch), dim3(kCpChunk), 0, h->stream, a, tr,
                           b, h->cp_rng + run->off, run->L0, run->L1, up);
        k += run->L1 - run->L0;
        continue;
      }
      if (wide(L)) {
        const int n = lo[L + 1] - lo[L];
        hipLaunchKernelGGL(k_cp_level, dim3(grid_of(n, 256)), dim3(256), 0, h->stream, a, tr, b,
                           lo[L], lo[L + 1], up);
        ++k;
        continue;
      }
      // (a narrow run ends at a wide level or where a chunked run starts)
      auto run_at = [&](int Lq) {
        if (wmax != 1024) return false;
        for (const auto& r : h->cp_runs)
          if (up ? Lq == r.L1 - 1 : Lq == r.L0) return true;
        return false;
      };
      int k1 = k;
      while (k1 < nl && !wide(up ? nl - 1 - k1 : k1) && (k1 == k || !run_at(up ? nl - 1 - k1 : k1)))
        ++k1;
      const int La = up ? nl - k1 : k, Lb = up ? nl - k : k1;  // levels [La, Lb)
      // (the pipelined kernel: records, at most 1024 nodes per level and kCpPipeLv levels)
      bool pipe = tr.rec != nullptr && Lb - La <= kCpPipeLv && cp_pipe_on();
      for (int L = La; L < Lb && pipe; ++L) pipe = lo[L + 1] - lo[L] <= 1024 && h->cp_lev_full[L];
      if (pipe)
        hipLaunchKernelGGL(k_cp_nodes_rec, dim3(1), dim3(1024), 0, h->stream, a, tr, b,
                           (const int*)nullptr, La, Lb, up);
      else
        hipLaunchKernelGGL(k_cp_nodes, dim3(1), dim3(1024), 0, h->stream, a, tr, b, La, Lb, up);
      k = k1;
    }
  }
}

int fe_cp_solve(nx_network* h, double rtol, int32_t* iters, double* relres, int32_t* converged) {
  CHECK(flush_assembly(h));
  // several ranks: the edge kernels over this rank's edges (se by global edge), the node
  // kernels over the summed blocks and node rhs (an: nrow indexes nb), the rows it owns
  const bool ranks = h->cp_Eg > 0;
  const int64_t Ee = ranks ? h->cp_Eown : h->E;
  const CpArgs a{(int)h->N, h->cp_k, h->cp_m, h->cp_nI, Ee, h->edge_R, h->fe_cellh, h->cp_cst,
                 h->cp_tI, h->cp_eb, ranks ? h->cp_nrowx : h->cp_nrow, h->cp_fac, h->cp_se,
                 h->cp_xn, ranks ? h->cp_gid : nullptr};
  CpArgs an = a;
  an.nrow = h->cp_nrow;
  double* nb = h->cp_se + 20 * h->cp_Eg;
  const int64_t nsum = 20 * h->cp_Eg + 2 * (int64_t)h->cp_nn;
  nx_network* hs[1] = {h};
  const Team t{hs, 1, nullptr};
  const CpTree tr{h->cp_nn, h->cp_nlev, h->cp_lev_off, h->cp_order, h->cp_inc_off, h->cp_inc,
                  h->cp_parent, h->cp_child_off, h->cp_child, h->cp_Pinv, h->cp_hv, h->cp_rec,
                  h->cp_rec ? h->cp_ctr : nullptr};
  const int nrb = grid_of(h->n_own, kRowsPerBlock * res_chunks(h->n_own));
  // (one thread per edge: 64-thread workgroups spread the edges over every CU. Staging the
  // edges' rows of b in LDS was measured slower, r06zd; the back-substitution's x rows go
  // out through LDS when they fit 64 KB, NXHIP_CP_XS=0 off)
  const int eb = std::max(1, grid_of(Ee, 64));
  const int per_e = h->cp_k * (int)h->N + 1 + h->cp_m * (int)h->N - 1;
  const char* xs_env = std::getenv("NXHIP_CP_XS");
  const size_t xs_lds = (xs_env == nullptr || std::atoi(xs_env) != 0) &&
                                (size_t)64 * per_e * sizeof(double) <= 64 * 1024
                            ? (size_t)64 * per_e * sizeof(double)
                            : 0;
  MrState s{};
  int pass = 0;
  h->last_dir_path = 4;  // the node-condensed route (nx_get_direct_path)
  for (; pass < 3; ++pass) {
    const double* b = pass ? h->tmp : h->rhs;  // refinement: the residual the check kept
    if (ranks) HIPCALL(hipMemsetAsync(h->cp_se, 0, sizeof(double) * nsum, h->stream));
    hipLaunchKernelGGL(k_cp_edge, dim3(eb), dim3(64), 0, h->stream, a, b);
    if (ranks) {
      hipLaunchKernelGGL(k_cp_nb, dim3(grid_of(2 * (int64_t)h->cp_nn, 256)), dim3(256), 0,
                         h->stream, h->cp_nrowx, h->cp_nn, b, nb);
      CHECK(team_allreduce(t, -5, (int)nsum));
    }
    cp_nodes_launch(h, ranks ? an : a, tr, ranks ? nb : b);
    hipLaunchKernelGGL(k_cp_back, dim3(eb), dim3(64), xs_lds, h->stream, a, b, h->x, h->cp_nown,
                       pass ? 1 : 0, xs_lds > 0 ? 1 : 0);
    if (ranks)
      CHECK(fe_true_residual_team(h, rtol, nrb));
    else
      fe_true_residual(h, rtol, nrb);
    HIPCALL(hipGetLastError());
    h->seq += 1;
    CHECK(wait_published(h));
    s = *h->h_last;
    if (s.converged || s.relres != s.relres) break;
  }
  if (iters) *iters = std::min(pass, 2) + 1;
  if (relres) *relres = s.relres;
  if (converged) *converged = s.converged;
  return NX_OK;
}

int solve_team(const Team& t, double rtol, int32_t maxit, int32_t check_every, int32_t* iters,
               double* relres, int32_t* converged) {
  for (int r = 0; r < t.P; ++r) {
    nx_network* h = t.hs[r];
    if (!h->have_lhs || !h->have_rhs) return fail(NX_ERR_STATE, "assemble lhs and rhs before solve");
    if (h->pc != t.hs[0]->pc) return fail(NX_ERR_STATE, "ranks disagree on the preconditioner");
  }
  if (maxit < 1) return fail(NX_ERR_ARG, "maxit must be >= 1");
  if (check_every < 2) check_every = 2;
  for (int r = 0; r < t.P; ++r) t.hs[r]->last_solver = 0;
  if (team_multi(t)) {  // every rank must take the same path (the signature holds it)
    CHECK(set_device(t.hs[0]));
    CHECK(check_schedules(t));
  }
  if (t.P == 1 && t.hs[0]->fe && (t.hs[0]->fe_aux || t.hs[0]->fe_cp) && t.hs[0]->solver == 1) {
    CHECK(set_device(t.hs[0]));
    int32_t conv = 0;
    CHECK(t.hs[0]->fe_cp ? fe_cp_solve(t.hs[0], rtol, iters, relres, &conv)
                         : fe_solve_direct(t.hs[0], rtol, iters, relres, &conv));
    if (conv) {
      t.hs[0]->last_solver = 1;
      if (converged) *converged = 1;
      return NX_OK;
    }
  }
  if (direct_applicable(t)) {
    CHECK(set_device(t.hs[0]));
    int32_t conv = 0;
    CHECK(solve_direct(t, rtol, iters, relres, &conv));
    if (conv) {
      for (int r = 0; r < t.P; ++r) t.hs[r]->last_solver = 1;
      if (converged) *converged = 1;
      return NX_OK;
    }
    // residual above rtol after a refinement step: MINRES from scratch
  }
  for (int r = 0; r < t.P; ++r) {  // MINRES: no deferred work, the lumped mass formed
    CHECK(flush_assembly(t.hs[r]));
    CHECK(ensure_dq(t.hs[r]));
  }
  if (check_every & 1) ++check_every;
  CHECK(set_device(t.hs[0]));
  const bool multi = team_multi(t);
  if (multi) CHECK(check_schedules(t));
  const bool lean_env = lean_mode();
  {  // one graph per solve (profiling and the all-reduce beta^2 variant keep the general path)
    nx_network* h0 = t.hs[0];
    const bool prof = h0->prof && t.g == nullptr;
    const bool ok_multi = !multi || (h0->beta_p2p && (!proc_rank(h0) || h0->rccl_graph_ok));
    if (h0->pc && !prof && lean_env && ok_multi) {
      const int rc = solve_lean(t, rtol, maxit, check_every, iters, relres, converged);
      if (rc != NX_ERR_RCCL || !proc_rank(h0)) return rc;  // RCCL capture refused: eager below
    }
  }
  for (int r = 0; r < t.P; ++r) t.hs[r]->pa.fuse_pack = 0;  // the general path packs itself
  hipStream_t s = t.hs[0]->stream;
  // r1 = r2 = b, w1 = w2 = x = 0
  for (int r = 0; r < t.P; ++r) {
    nx_network* h = t.hs[r];
    const int64_t n = h->n_own;
    for (int i = 0; i < 2; ++i) {
      if (n > 0)
        HIPCALL(hipMemcpyAsync(h->vb[i], h->rhs, sizeof(double) * n, hipMemcpyDeviceToDevice, h->stream));
      if (h->n_ghost > 0) HIPCALL(hipMemsetAsync(h->vb[i] + n, 0, sizeof(double) * h->n_ghost, h->stream));
      if (n > 0) HIPCALL(hipMemsetAsync(h->wb[i], 0, sizeof(double) * n, h->stream));
    }
    HIPCALL(hipMemsetAsync(h->x, 0, sizeof(double) * h->n_col, h->stream));
  }
  if (t.hs[0]->pc) {  // beta_1^2 = b . P^{-1} b
    // the flags of the iterations (mode-1 kernels ignore them, except that the start's down
    // sweep builds G when the dense top is on)
    for (int r = 0; r < t.P; ++r) {
      nx_network* h = t.hs[r];
      h->pa.factored = h->pa.dc_kappa ? 1 : 0;
      h->pa.mdense =
          (multi && h->pa.dense && h->pa.KJ && h->pa.n_coarse > 0 && h->pa.lin) ? 1 : 0;
    }
    CHECK(team_pc(t, 0, 1));
    for (int r = 0; r < t.P; ++r) {  // coefficients of this assembly's D (fixed per solve)
      nx_network* h = t.hs[r];
      // k_pc_down_lds (start) did factor + G (+ KJ, roots and weights with several ranks)
      const bool fused = h->pc_lds && h->pc_jobs > 0 && (!multi || h->pa.fused);
      if (h->pa.dc_kappa && !fused) {
        const int nmax = (int)std::max<int64_t>(h->pc_ndc, h->pc_slots);
        if (nmax > 0)
          hipLaunchKernelGGL(k_pc_factor, dim3(grid_of(nmax, 256)), dim3(256), 0, h->stream,
                             h->pa, (int)h->pc_ndc, (int)h->pc_slots);
      }
      const bool md = multi && h->pa.dense && h->pa.KJ && h->pa.n_coarse > 0 && h->pa.lin;
      if (h->pa.dense && (md || !multi) && !fused)
        hipLaunchKernelGGL(k_pc_gbuild, dim3(h->pa.n_top), dim3(64), 0, h->stream, h->pa);
      if (md && !fused) hipLaunchKernelGGL(k_pc_wroot, dim3(1), dim3(kTopThreads), 0, h->stream, h->pa);
    }
  } else {
    for (int r = 0; r < t.P; ++r) {
      nx_network* h = t.hs[r];
      hipLaunchKernelGGL(k_sumsq, dim3(h->nB), dim3(kBlock), 0, h->stream, h->rhs, h->n_own, h->partB);
    }
  }
  if (multi) CHECK(team_reduce_slot(t, false, 2));
  for (int r = 0; r < t.P; ++r) {
    nx_network* h = t.hs[r];
    for (int b = 0; b < 2; ++b) {  // both state buffers start identical
      if (multi)
        hipLaunchKernelGGL(k_mr_init<true>, dim3(1), dim3(kBlock), 0, h->stream, h->partB, nB_of(h),
                           h->red, h->st + b, rtol, maxit);
      else
        hipLaunchKernelGGL(k_mr_init<false>, dim3(1), dim3(kBlock), 0, h->stream, h->partB,
                           nB_of(h), h->red, h->st + b, rtol, maxit);
    }
  }
  HIPCALL(hipGetLastError());

  // Chunks of check_every iterations, one host check each: a HIP graph, except with RCCL
  // (eager launches) and when profiling (an event pair around every k_mr_a of a chunk;
  // after the check only the launches that ran a Lanczos step are added).
  nx_network* h0 = t.hs[0];
  const bool prof = h0->prof && t.g == nullptr;
  // RCCL iterations are captured too (host-side enqueue of ~8 operations per iteration
  // would otherwise pace the loop); if the capture fails, that handle stays eager
  const bool rccl = proc_rank(t.hs[0]);
  bool use_graph = !prof && (!rccl || h0->rccl_graph_ok);
  if (use_graph) {
    const int rc = build_chunk_graph(t, check_every);
    if (rc != NX_OK) {
      if (!rccl) return rc;
      (void)hipGetLastError();
      (void)drop_graph(graph_slot(t));
      h0->rccl_graph_ok = false;
      use_graph = false;
    }
  }
  h0->last_graph = use_graph;
  if (prof && (int)h0->ev_pool.size() < 2 * check_every) {
    for (auto& e : h0->ev_pool) (void)hipEventDestroy(e);
    h0->ev_pool.assign(2 * check_every, nullptr);
    for (auto& e : h0->ev_pool) HIPCALL(hipEventCreate(&e));
  }
  int64_t launched = 0;
  int nb_before = 0;
  const MrState* last = nullptr;
  for (;;) {
    if (use_graph) {
      HIPCALL(hipGraphLaunch(*graph_slot(t).exec, s));
    } else {
      h0->prof_k = 0;
      for (int j = 0; j < check_every; ++j) CHECK(launch_iteration(t, launched + j + 1));
    }
    launched += check_every;
    for (int r = 0; r < t.P; ++r)
      HIPCALL(hipMemcpyAsync(t.hs[r]->h_st, t.hs[r]->st, 2 * sizeof(MrState), hipMemcpyDeviceToHost,
                             t.hs[r]->stream));
    HIPCALL(hipStreamSynchronize(s));
    // the chunk ends with k even -> S[0] is the latest; once the solve stopped, k_mr_b
    // has made both buffers identical
    last = &h0->h_st[0];
    for (int r = 1; r < t.P; ++r) {  // the ranks run the same recurrence on the same scalars
      const MrState& o = t.hs[r]->h_st[0];
      if (o.it != last->it || o.done != last->done || o.relres != last->relres) {
        char msg[256];
        std::snprintf(msg, sizeof(msg),
                      "ranks diverged: rank %d it %d done %d relres %.17g beta %.17g alfa %.17g "
                      "vs rank 0 it %d done %d relres %.17g beta %.17g alfa %.17g",
                      r, o.it, o.done, o.relres, o.beta, o.alfa, last->it, last->done,
                      last->relres, last->beta, last->alfa);
        return fail(NX_ERR_STATE, msg);
      }
    }
    if (prof) {
      const int ran = last->nb - nb_before;
      for (int j = 0; j < ran && j < h0->prof_k; ++j) {
        float ms = 0.f;
        HIPCALL(hipEventElapsedTime(&ms, h0->ev_pool[2 * j], h0->ev_pool[2 * j + 1]));
        h0->spmv_ms += ms;
        h0->spmv_cnt += 1;
      }
      nb_before = last->nb;
    }
    if (last->done) break;
  }
  if (iters) *iters = last->it;
  if (relres) *relres = last->relres;
  if (converged) *converged = last->converged;
  return NX_OK;
}

}  // namespace

NX_API int nx_solve(nx_network_t* h, double rtol, int32_t maxit, int32_t check_every,
                    int32_t* iters, double* relres, int32_t* converged) {
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (h->group) return fail(NX_ERR_STATE, "the handle belongs to a group: use nx_group_solve");
  nx_network* hs[1] = {h};
  return solve_team(Team{hs, 1, nullptr}, rtol, maxit, check_every, iters, relres, converged);
}

NX_API int nx_get_solution(nx_network_t* h, double* xo) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h || !xo) return fail(NX_ERR_ARG, "null argument");
  CHECK(set_device(h));
  HIPCALL(hipMemcpyAsync(xo, h->x, sizeof(double) * h->n_own, hipMemcpyDeviceToHost, h->stream));
  HIPCALL(hipStreamSynchronize(h->stream));
  return NX_OK;
}

NX_API int nx_set_output_map(nx_network_t* h, int64_t n, const int32_t* rows) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h || (n > 0 && !rows)) return fail(NX_ERR_ARG, "null argument");
  if (n != h->n_own) return fail(NX_ERR_ARG, "the output map must list every owned row once");
  std::vector<char> seen((size_t)n, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (rows[i] < 0 || rows[i] >= n || seen[(size_t)rows[i]])
      return fail(NX_ERR_ARG, "the output map is not a permutation of the owned rows");
    seen[(size_t)rows[i]] = 1;
  }
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  if (h->out_idx) HIPCALL(hipFree(h->out_idx));
  h->out_idx = nullptr;
  h->n_out = 0;
  if (n > 0) {
    HIPCALL(hipMalloc((void**)&h->out_idx, sizeof(int) * n));
    HIPCALL(hipMemcpy(h->out_idx, rows, sizeof(int) * n, hipMemcpyHostToDevice));
  }
  h->n_out = n;
  return NX_OK;
}

NX_API int nx_get_solution_blocks(nx_network_t* h, double* out) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h || !out) return fail(NX_ERR_ARG, "null argument");
  if (!h->out_idx && h->n_own > 0) return fail(NX_ERR_STATE, "nx_set_output_map first");
  CHECK(set_device(h));
  if (h->n_own > 0) {
    // tmp (n_col >= n_own) is free outside nx_solve / nx_spmv_host
    hipLaunchKernelGGL(k_gather_out, dim3(grid_of(h->n_own, kBlock)), dim3(kBlock), 0, h->stream,
                       h->x, h->out_idx, h->n_own, h->tmp);
    HIPCALL(hipGetLastError());
    HIPCALL(hipMemcpyAsync(out, h->tmp, sizeof(double) * h->n_own, hipMemcpyDeviceToHost,
                           h->stream));
  }
  HIPCALL(hipStreamSynchronize(h->stream));
  return NX_OK;
}

constexpr int kMaxSnap = 64;

NX_API int nx_snapshot_solution(nx_network_t* h, int32_t slot) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (slot < 0 || slot >= kMaxSnap) return fail(NX_ERR_ARG, "snapshot slot out of range");
  if (!h->out_idx && h->n_own > 0) return fail(NX_ERR_STATE, "nx_set_output_map first");
  CHECK(set_device(h));
  if ((int)h->snap.size() <= slot) {
    h->snap.resize((size_t)slot + 1, nullptr);
    h->snap_ev.resize((size_t)slot + 1, nullptr);
  }
  if (!h->snap_ev[slot]) HIPCALL(hipEventCreateWithFlags(&h->snap_ev[slot], hipEventDisableTiming));
  if (h->n_own > 0) {
    if (!h->snap[slot]) CHECK(dalloc(&h->snap[slot], h->n_own));
    hipLaunchKernelGGL(k_gather_out, dim3(grid_of(h->n_own, kBlock)), dim3(kBlock), 0, h->stream,
                       h->x, h->out_idx, h->n_own, h->snap[slot]);
    HIPCALL(hipGetLastError());
  }
  HIPCALL(hipEventRecord(h->snap_ev[slot], h->stream));
  return NX_OK;
}

NX_API int nx_fetch_snapshot(nx_network_t* h, int32_t slot, double* out) {
  if (!h || !out) return fail(NX_ERR_ARG, "null argument");
  if (slot < 0 || slot >= (int)h->snap_ev.size() || !h->snap_ev[slot])
    return fail(NX_ERR_STATE, "no snapshot in this slot (nx_snapshot_solution first)");
  CHECK(set_device(h));
  if (h->n_own > 0) {
    if (!h->copy_stream) HIPCALL(hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking));
    HIPCALL(hipStreamWaitEvent(h->copy_stream, h->snap_ev[slot], 0));
    HIPCALL(hipMemcpyAsync(out, h->snap[slot], sizeof(double) * h->n_own, hipMemcpyDeviceToHost,
                           h->copy_stream));
    HIPCALL(hipStreamSynchronize(h->copy_stream));
  }
  return NX_OK;
}

NX_API int nx_host_alloc(int64_t bytes, void** out) {
  if (!out || bytes < 0) return fail(NX_ERR_ARG, "bad argument");
  *out = nullptr;
  if (bytes == 0) return NX_OK;
  HIPCALL(hipHostMalloc(out, (size_t)bytes, hipHostMallocDefault));
  return NX_OK;
}

NX_API int nx_host_free(void* p) {
  if (p) HIPCALL(hipHostFree(p));
  return NX_OK;
}

NX_API int nx_get_vector(nx_network_t* h, int32_t which, double* out) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h || !out) return fail(NX_ERR_ARG, "null argument");
  CHECK(set_device(h));
  const double* src = which == 0 ? h->x : which == 1 ? h->rhs : which == 2 ? h->z : nullptr;
  if (!src) return fail(NX_ERR_ARG, "which: 0 = solution, 1 = rhs, 2 = preconditioned residual");
  HIPCALL(hipMemcpyAsync(out, src, sizeof(double) * h->n_own, hipMemcpyDeviceToHost, h->stream));
  HIPCALL(hipStreamSynchronize(h->stream));
  return NX_OK;
}

NX_API int nx_get_rhs(nx_network_t* h, double* b) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h || !b) return fail(NX_ERR_ARG, "null argument");
  CHECK(set_device(h));
  HIPCALL(hipMemcpyAsync(b, h->rhs, sizeof(double) * h->n_own, hipMemcpyDeviceToHost, h->stream));
  HIPCALL(hipStreamSynchronize(h->stream));
  return NX_OK;
}

NX_API int nx_get_csr(nx_network_t* h, int32_t* rowptr, int32_t* col, double* val) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  CHECK(set_device(h));
  if (rowptr)
    HIPCALL(hipMemcpyAsync(rowptr, h->rowptr, sizeof(int) * (h->n_own + 1), hipMemcpyDeviceToHost,
                           h->stream));
  if (col)
    HIPCALL(hipMemcpyAsync(col, h->col, sizeof(int) * h->nnz, hipMemcpyDeviceToHost, h->stream));
  if (val)
    HIPCALL(hipMemcpyAsync(val, h->val, sizeof(double) * h->nnz, hipMemcpyDeviceToHost, h->stream));
  HIPCALL(hipStreamSynchronize(h->stream));
  return NX_OK;
}

NX_API int nx_spmv_host(nx_network_t* h, const double* xh, double* yh) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h || !xh || !yh) return fail(NX_ERR_ARG, "null argument");
  if (!h->have_lhs) return fail(NX_ERR_STATE, "assemble the matrix first");
  CHECK(set_device(h));
  HIPCALL(hipMemcpyAsync(h->tmp, xh, sizeof(double) * h->n_col, hipMemcpyHostToDevice, h->stream));
  // dedicated output buffer: the Krylov vectors keep their state
  double* y = nullptr;
  HIPCALL(hipMallocAsync((void**)&y, sizeof(double) * std::max<int64_t>(h->n_own, 1), h->stream));
  if (h->nblk > 0)
    hipLaunchKernelGGL(k_spmv, dim3(h->nblk), dim3(kBlock), 0, h->stream, csr_of(h), h->tmp, y);
  HIPCALL(hipGetLastError());
  HIPCALL(hipMemcpyAsync(yh, y, sizeof(double) * h->n_own, hipMemcpyDeviceToHost, h->stream));
  HIPCALL(hipFreeAsync(y, h->stream));
  HIPCALL(hipStreamSynchronize(h->stream));
  return NX_OK;
}

NX_API int nx_true_residual(nx_network_t* h, double* relres) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h || !relres) return fail(NX_ERR_ARG, "null argument");
  if (!h->have_lhs || !h->have_rhs) return fail(NX_ERR_STATE, "assemble first");
  if (h->group) return fail(NX_ERR_STATE, "group member: compute the residual from the solutions");
  CHECK(set_device(h));
  {
    nx_network* hs[1] = {h};
    CHECK(team_halo(Team{hs, 1, nullptr}, VS_X, 0));
  }
  hipLaunchKernelGGL(k_residual, dim3(h->nblk), dim3(kBlock), 0, h->stream, csr_of(h), h->x,
                     h->rhs, h->partials, h->nblk, nullptr);
  double* d = h->red + 2;  // slots 2, 3 are free outside nx_solve
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kReduceThreads), 0, h->stream, h->partials, h->nblk, d);
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kReduceThreads), 0, h->stream, h->partials + h->nblk,
                     h->nblk, d + 1);
  HIPCALL(hipGetLastError());
  if (h->hcomm) CHECK(hc_allreduce(h, d, 2, 0));
  if (h->comm) NCCLCALL(ncclAllReduce(d, d, 2, ncclDouble, ncclSum, h->comm, h->stream));
  HIPCALL(hipStreamSynchronize(h->stream));
  double hd[2] = {0.0, 0.0};
  HIPCALL(hipMemcpy(hd, d, sizeof(hd), hipMemcpyDeviceToHost));
  *relres = hd[1] > 0 ? std::sqrt(hd[0] / hd[1]) : std::sqrt(hd[0]);
  return NX_OK;
}

NX_API int nx_sync(nx_network_t* h) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  return NX_OK;
}

NX_API int nx_set_profiling(nx_network_t* h, int32_t enable) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  h->prof = enable != 0;
  return NX_OK;
}

NX_API int nx_get_profile(nx_network_t* h, double* spmv_ms, int64_t* spmv_count, double* asm_ms,
                          int64_t* asm_count) {
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (spmv_ms) *spmv_ms = h->spmv_ms;
  if (spmv_count) *spmv_count = h->spmv_cnt;
  if (asm_ms) *asm_ms = h->asm_ms;
  if (asm_count) *asm_count = h->asm_cnt;
  return NX_OK;
}

NX_API int nx_get_profile_direct(nx_network_t* h, double* ms4, int64_t* count) {
  if (!h || !ms4) return fail(NX_ERR_ARG, "null argument");
  for (int k = 0; k < 4; ++k) ms4[k] = h->dir_ms[k];
  if (count) *count = h->dir_cnt;
  return NX_OK;
}

NX_API int nx_get_direct_info(nx_network_t* h, int32_t* fused, int32_t* n_left) {
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (fused) *fused = h->fres_ok ? 1 : 0;
  if (n_left) *n_left = h->n_left;
  return NX_OK;
}

NX_API int nx_get_direct_path(nx_network_t* h, int32_t* path) {
  if (!h || !path) return fail(NX_ERR_ARG, "null argument");
  *path = h->last_dir_path;
  return NX_OK;
}

NX_API int nx_get_direct_sup(nx_network_t* h, int32_t* sup) {
  if (!h || !sup) return fail(NX_ERR_ARG, "null argument");
  *sup = h->last_sup ? 1 : 0;
  return NX_OK;
}

NX_API int nx_debug_set_wait_polls(nx_network_t* h, uint32_t polls) {
  if (!h) return fail(NX_ERR_ARG, "null handle");
  h->dstep_polls = polls;
  return NX_OK;
}

NX_API int nx_reset_profile(nx_network_t* h) {
  if (!h) return fail(NX_ERR_ARG, "null handle");
  h->spmv_ms = h->asm_ms = 0.0;
  h->spmv_cnt = h->asm_cnt = 0;
  for (double& v : h->dir_ms) v = 0.0;
  h->dir_cnt = 0;
  return NX_OK;
}

NX_API int nx_bench_spmv(nx_network_t* h, int32_t reps, double* ms_per_spmv) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h || !ms_per_spmv || reps < 1) return fail(NX_ERR_ARG, "bad argument");
  if (!h->have_lhs) return fail(NX_ERR_STATE, "assemble the matrix first");
  CHECK(set_device(h));
  if (h->nblk == 0) {
    *ms_per_spmv = 0.0;
    return NX_OK;
  }
  // x = rhs-sized data already resident: use vb[0] as input, tmp as output
  hipLaunchKernelGGL(k_spmv, dim3(h->nblk), dim3(kBlock), 0, h->stream, csr_of(h), h->vb[0], h->tmp);
  HIPCALL(hipEventRecord(h->ev[0], h->stream));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL(k_spmv, dim3(h->nblk), dim3(kBlock), 0, h->stream, csr_of(h), h->vb[0],
                       h->tmp);
  HIPCALL(hipEventRecord(h->ev[1], h->stream));
  HIPCALL(hipEventSynchronize(h->ev[1]));
  HIPCALL(hipGetLastError());
  float ms = 0.f;
  HIPCALL(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
  *ms_per_spmv = ms / reps;
  return NX_OK;
}


NX_API int nx_get_graph_mode(nx_network_t* h, int32_t* graph) {
  if (!h || !graph) return fail(NX_ERR_ARG, "null argument");
  *graph = h->last_graph ? 1 : 0;
  return NX_OK;
}

NX_API int nx_bench_spmv_cold(nx_network_t* h, int32_t reps, int32_t* copies_out,
                              double* ms_per_spmv) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h || !ms_per_spmv || reps < 1) return fail(NX_ERR_ARG, "bad argument");
  if (!h->have_lhs) return fail(NX_ERR_STATE, "assemble the matrix first");
  CHECK(set_device(h));
  if (h->nblk == 0) {
    *ms_per_spmv = 0.0;
    return NX_OK;
  }
  // enough private copies of (rowptr, col, val, x, y) that a rotation touches > 512 MiB,
  // twice the 256 MiB Infinity Cache: every SpMV streams its operands from HBM
  const size_t bytes = sizeof(int) * (h->n_own + 1) + sizeof(int) * h->nnz +
                       sizeof(double) * h->nnz + sizeof(double) * (h->n_col + h->n_own);
  const int K = (int)std::min<size_t>(64, std::max<size_t>(2, (512ull << 20) / bytes + 1));
  std::vector<void*> bufs;
  auto release = [&]() {
    for (void* p : bufs) (void)hipFree(p);
  };
  std::vector<Csr> mats(K);
  std::vector<double*> xs(K), ys(K);
  for (int i = 0; i < K; ++i) {
    int *rp = nullptr, *cl = nullptr;
    double *vl = nullptr, *x = nullptr, *y = nullptr;
    if (hipMalloc((void**)&rp, sizeof(int) * (h->n_own + 1)) != hipSuccess ||
        hipMalloc((void**)&cl, sizeof(int) * h->nnz) != hipSuccess ||
        hipMalloc((void**)&vl, sizeof(double) * h->nnz) != hipSuccess ||
        hipMalloc((void**)&x, sizeof(double) * h->n_col) != hipSuccess ||
        hipMalloc((void**)&y, sizeof(double) * h->n_own) != hipSuccess) {
      for (void* p : {(void*)rp, (void*)cl, (void*)vl, (void*)x, (void*)y})
        if (p) bufs.push_back(p);
      release();
      return fail(NX_ERR_HIP, "cold SpMV buffers: out of device memory");
    }
    for (void* p : {(void*)rp, (void*)cl, (void*)vl, (void*)x, (void*)y}) bufs.push_back(p);
    (void)hipMemcpyAsync(rp, h->rowptr, sizeof(int) * (h->n_own + 1), hipMemcpyDeviceToDevice, h->stream);
    (void)hipMemcpyAsync(cl, h->col, sizeof(int) * h->nnz, hipMemcpyDeviceToDevice, h->stream);
    (void)hipMemcpyAsync(vl, h->val, sizeof(double) * h->nnz, hipMemcpyDeviceToDevice, h->stream);
    (void)hipMemcpyAsync(x, h->vb[0], sizeof(double) * h->n_col, hipMemcpyDeviceToDevice, h->stream);
    mats[i] = Csr{rp, cl, vl, h->n_own};
    xs[i] = x;
    ys[i] = y;
  }
  for (int i = 0; i < K; ++i)  // warm the code path, then rotate
    hipLaunchKernelGGL(k_spmv, dim3(h->nblk), dim3(kBlock), 0, h->stream, mats[i], xs[i], ys[i]);
  hipEvent_t e0 = h->ev[0], e1 = h->ev[1];
  int rc = NX_OK;
  if (hipEventRecord(e0, h->stream) != hipSuccess) rc = fail(NX_ERR_HIP, "event record failed");
  for (int r = 0; r < reps && rc == NX_OK; ++r) {
    const int i = r % K;
    hipLaunchKernelGGL(k_spmv, dim3(h->nblk), dim3(kBlock), 0, h->stream, mats[i], xs[i], ys[i]);
  }
  float ms = 0.f;
  if (rc == NX_OK && (hipEventRecord(e1, h->stream) != hipSuccess ||
                      hipEventSynchronize(e1) != hipSuccess ||
                      hipEventElapsedTime(&ms, e0, e1) != hipSuccess))
    rc = fail(NX_ERR_HIP, "cold SpMV timing failed");
  (void)hipStreamSynchronize(h->stream);
  release();
  if (rc != NX_OK) return rc;
  *ms_per_spmv = ms / reps;
  if (copies_out) *copies_out = K;
  return NX_OK;
}

namespace {
void free_cycles(nx_network* h);
}  // namespace

NX_API int nx_set_preconditioner(nx_network_t* h, int32_t enable, int64_t n_chains,
                                 const int32_t* chain_edge, const int32_t* chain_flip,
                                 const int32_t* chain_up, const int32_t* chain_lo, int64_t n_slots,
                                 const int32_t* slot_lam, const int32_t* slot_pchain,
                                 const int32_t* slot_parent, const int32_t* slot_dc_off,
                                 const int32_t* slot_dc, const int32_t* dc_lo,
                                 const int32_t* slot_plam, int32_t n_jobs,
                                 const int32_t* job_chain_off, const int32_t* job_lvl_off,
                                 int32_t n_lvl, const int32_t* lvl_slot_off, int32_t n_top_lvl,
                                 const int32_t* top_lvl_off) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  h->sched_checked = false;
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  CHECK(drop_handle_graphs(h));  // captured launches depend on the preconditioner
  free_cycles(h);  // (nx_set_cycles belongs to this decomposition: set again after it)
  if (!enable) {
    h->pc = false;
    return NX_OK;
  }
  if (h->fe)
    return fail(NX_ERR_STATE, "the tree preconditioner needs the P1/DG0 layout (nx_create)");
  const int N = h->N;
  int variant;
  if (N <= 16) variant = 5;  // 8 lanes x 2 cells: one chain round per job (swept: 16x1 +8%)
  // (N <= 32 by 8 lanes x 4 cells, 128 chains per pass: slower, 8-rank C4 rehearsal r03o --
  // team up 50 -> 57 us, down 41 -> 66 us per rank; the lanes' serial work dominates)
  else if (N <= 32) variant = 1;
  else if (N <= 64) variant = 2;
  else if (N <= 128) variant = 3;
  else if (N <= 256) variant = 4;
  else if (N <= 512) variant = 8;
  else if (N <= 1024) variant = 9;
  else return fail(NX_ERR_ARG, "tree preconditioner supports N <= 1024 cells per edge");
  if (n_chains != h->E) return fail(NX_ERR_ARG, "one chain per local edge expected");
  // one slot per owned multiplier, plus (several ranks) the ghost junctions at the ends of
  // local edges, which are coarse (nx_set_coarse)
  if (n_slots < h->B || n_slots > h->B + h->n_ghost)
    return fail(NX_ERR_ARG, "one junction slot per owned multiplier (+ ghost junctions) expected");
  if (n_jobs < 0 || n_lvl < 0 || n_top_lvl < 0) return fail(NX_ERR_ARG, "negative sizes");
  if (h->E > 0 && n_jobs < 1) return fail(NX_ERR_ARG, "chains need at least one job");
  for (int64_t c = 0; c < n_chains; ++c) {
    if (chain_edge[c] < 0 || chain_edge[c] >= h->E) return fail(NX_ERR_ARG, "chain_edge out of range");
    if (chain_up[c] < -1 || chain_up[c] >= n_slots || chain_lo[c] < -1 || chain_lo[c] >= n_slots)
      return fail(NX_ERR_ARG, "chain end slot out of range");
  }
  for (int64_t j = 0; j < n_slots; ++j) {
    if (slot_lam[j] < h->n_edge_dofs || slot_lam[j] >= h->n_col ||
        (slot_lam[j] >= h->n_own && h->nranks == 1))
      return fail(NX_ERR_ARG, "slot_lam must be a multiplier row or ghost column");
    if (slot_pchain[j] < -1 || slot_pchain[j] >= n_chains || slot_parent[j] < -1 ||
        slot_parent[j] >= n_slots)
      return fail(NX_ERR_ARG, "slot parent out of range");
  }
  for (int64_t i = 0; i < (n_slots > 0 ? slot_dc_off[n_slots] : 0); ++i)
    if (slot_dc[i] < 0 || slot_dc[i] >= n_chains || dc_lo[i] != chain_lo[slot_dc[i]])
      return fail(NX_ERR_ARG, "slot_dc / dc_lo inconsistent");
  if (job_chain_off[0] != 0 || job_chain_off[n_jobs] != n_chains)
    return fail(NX_ERR_ARG, "job_chain_off must cover all chains");
  if (job_lvl_off[n_jobs] != n_lvl) return fail(NX_ERR_ARG, "job_lvl_off must end at n_lvl");
  if (n_slots > 0 && (int64_t)(n_lvl > 0 ? lvl_slot_off[n_lvl] : 0) +
                             (top_lvl_off[n_top_lvl] - top_lvl_off[0]) != n_slots)
    return fail(NX_ERR_ARG, "levels must cover all slots");
  for (void* p : h->pc_bufs) (void)hipFree(p);
  h->pc_bufs.clear();
  auto up = [&](const int32_t* src, int64_t n) -> const int* {
    int* d = nullptr;
    if (n <= 0) n = 1;
    if (hipMalloc((void**)&d, sizeof(int) * n) != hipSuccess) return nullptr;
    h->pc_bufs.push_back(d);
    if (src && hipMemcpy(d, src, sizeof(int) * n, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return d;
  };
  auto scratch = [&](int64_t n) -> double* {
    double* d = nullptr;
    if (n <= 0) n = 1;
    if (hipMalloc((void**)&d, sizeof(double) * n) != hipSuccess) return nullptr;
    h->pc_bufs.push_back(d);
    return d;
  };
  PcArgs pa{};
  pa.N = N;
  pa.invN = 1.0 / (double)N;
  pa.chain_edge = up(chain_edge, n_chains);
  pa.chain_flip = up(chain_flip, n_chains);
  pa.chain_up = up(chain_up, n_chains);
  pa.chain_lo = up(chain_lo, n_chains);
  pa.slot_lam = up(slot_lam, n_slots);
  pa.slot_pchain = up(slot_pchain, n_slots);
  pa.slot_parent = up(slot_parent, n_slots);
  pa.slot_dc_off = up(slot_dc_off, n_slots + 1);
  pa.slot_dc = up(slot_dc, slot_dc_off[n_slots]);
  pa.dc_lo = up(dc_lo, slot_dc_off[n_slots]);
  pa.slot_plam = up(slot_plam, n_slots);
  pa.job_chain_off = up(job_chain_off, n_jobs + 1);
  pa.job_lvl_off = up(job_lvl_off, n_jobs + 1);
  pa.lvl_slot_off = up(lvl_slot_off, n_lvl + 1);
  pa.top_lvl_off = up(top_lvl_off, n_top_lvl + 1);
  pa.n_top_lvl = n_top_lvl;
  h->top_ts0 = top_lvl_off[0];
  h->top_nt = top_lvl_off[n_top_lvl] - top_lvl_off[0];
  pa.top_ts0 = h->top_ts0;
  pa.top_nt = h->top_nt;
  pa.top_dc0 = h->top_nt > 0 ? slot_dc_off[h->top_ts0] : 0;
  pa.top_ndc = h->top_nt > 0 ? slot_dc_off[h->top_ts0 + h->top_nt] - pa.top_dc0 : 0;
  pa.n_jobs = n_jobs;
  pa.n_dc_all = (int)slot_dc_off[n_slots];
  pa.n_slots_all = (int)n_slots;
  pa.dq = h->dq;
  pa.chain_T = scratch(n_chains);
  pa.chain_It = scratch(n_chains);
  pa.chain_Ib = scratch(n_chains);
  pa.slot_D = scratch(n_slots);
  pa.slot_J = scratch(n_slots);
  pa.slot_A = scratch(n_slots);
  pa.slot_B = scratch(n_slots);
  pa.slot_z = scratch(n_slots);
  pa.lin = 0;
  pa.dense = 0;
  pa.factored = 0;  // set by solve after k_pc_factor
  pa.mdense = 0;
  pa.KJ = nullptr;
  pa.dc_kappa = scratch(slot_dc_off[n_slots]);
  pa.slot_invD = scratch(n_slots);
  {  // consistent-mass flux block: pivots of T = tridiag(1, 4, 1), 2 at both ends
    const std::vector<double> ti = mass_lu(N);
    double* d = scratch((int64_t)ti.size());
    if (d == nullptr || hipMemcpy(d, ti.data(), sizeof(double) * ti.size(), hipMemcpyHostToDevice) !=
                            hipSuccess)
      return fail(NX_ERR_HIP, "preconditioner upload failed");
    pa.Tlu = d;
    pa.mo_div = 3.0;  // P1 (nx_set_cell_mass: a condensed (k, 0) system)
    h->cond_mass = false;
    pa.exact = 1;  // (nx_set_pc_exact(h, 0): lumped D, P = blockdiag(D, G^T D^{-1} G))
  }
  for (const void* p : {(const void*)pa.chain_edge, (const void*)pa.chain_flip, (const void*)pa.chain_up,
                        (const void*)pa.chain_lo, (const void*)pa.slot_lam, (const void*)pa.slot_pchain,
                        (const void*)pa.slot_parent, (const void*)pa.slot_dc_off, (const void*)pa.slot_dc,
                        (const void*)pa.job_chain_off, (const void*)pa.job_lvl_off,
                        (const void*)pa.lvl_slot_off, (const void*)pa.top_lvl_off,
                        (const void*)pa.chain_T, (const void*)pa.chain_It, (const void*)pa.chain_Ib,
                        (const void*)pa.slot_D, (const void*)pa.slot_J, (const void*)pa.dc_lo,
                        (const void*)pa.slot_plam, (const void*)pa.slot_A, (const void*)pa.slot_B,
                        (const void*)pa.slot_z})
    if (p == nullptr) return fail(NX_ERR_HIP, "preconditioner upload failed");
  if (!h->z) CHECK(dalloc(&h->z, std::max<int64_t>(h->n_col, 1)));
  if (!h->vv) CHECK(dalloc(&h->vv, std::max<int64_t>(h->n_own, 1)));
  {  // stored Lanczos vectors
    if (!h->vs) {
      CHECK(dalloc(&h->vs, (int64_t)kMaxV * std::max<int64_t>(h->n_own, 1)));
      CHECK(dalloc(&h->hist, 4 * (int64_t)kMaxV));
    }
  }
  HIPCALL(hipMemset(h->z, 0, sizeof(double) * std::max<int64_t>(h->n_col, 1)));
  if (n_jobs + 1 > h->nB) {  // partB holds one partial per job + the top block
    HIPCALL(hipFree(h->partB));
    h->partB = nullptr;
    h->nB = n_jobs + 1;
    CHECK(dalloc(&h->partB, h->nB));
  }
  // LDS kernels when every job (and the top part) fits their caps
  bool lds = (top_lvl_off[n_top_lvl] - top_lvl_off[0]) <= kCapT && n_top_lvl <= kMaxTopLvl;
  if (lds && n_top_lvl > 0 && top_lvl_off[n_top_lvl] > top_lvl_off[0])
    lds = slot_dc_off[top_lvl_off[n_top_lvl]] - slot_dc_off[top_lvl_off[0]] <= kCapTDC;
  for (int j = 0; lds && j < n_jobs; ++j) {
    if (job_chain_off[j + 1] - job_chain_off[j] > kCapC) lds = false;
    if (job_lvl_off[j + 1] > job_lvl_off[j]) {
      const int a = lvl_slot_off[job_lvl_off[j]], b = lvl_slot_off[job_lvl_off[j + 1]];
      if (b - a > kCapS || slot_dc_off[b] - slot_dc_off[a] > kCapDC) lds = false;
    }
  }
  if (const char* e = std::getenv("NXHIP_PC_GLOBAL")) lds = lds && std::atoi(e) == 0;
  lds = lds && !h->force_global;  // the ranks chose together (nx_set_pc_kernels)
  // fused residual of the direct solve (one rank, LDS kernels): a junction's multiplier row
  // is formed by its job's down sweep when its chains -- the parent chain (lo = j) and the
  // hanging ones (up = j) -- are exactly slot_pchain / slot_dc and all in that job; every
  // other multiplier row goes to k_dir_publish_fr (the top part's)
  pa.fres = 0;
  pa.edge_x = h->edge_x;
  pa.edge_R = h->edge_R;
  h->fres_ok = false;
  h->d_left = nullptr;
  h->n_left = 0;
  h->dstep_ok = false;  // (the fused step's buffers were in the freed pc_bufs)
  h->d_chain_post = h->d_left_off = nullptr;
  h->d_post = nullptr;
  h->d_dsync = nullptr;
  h->d_tsync = nullptr;
  h->dstep_epoch = 0;
  h->dstep_off = false;
  h->need_r = false;
  if (lds && n_jobs > 0) {  // one rank or several (then only owned rows of lower jobs)
    std::vector<int> job_of_chain(n_chains, -1), job_of_slot(n_slots, -1);
    for (int jb = 0; jb < n_jobs; ++jb) {
      for (int c = job_chain_off[jb]; c < job_chain_off[jb + 1]; ++c) job_of_chain[c] = jb;
      for (int lv = job_lvl_off[jb]; lv < job_lvl_off[jb + 1]; ++lv)
        for (int j = lvl_slot_off[lv]; j < lvl_slot_off[lv + 1]; ++j) job_of_slot[j] = jb;
    }
    std::vector<int> n_lo(n_slots, 0), n_up(n_slots, 0);
    std::vector<char> far(n_slots, 0);  // a chain at this junction lies in another job
    for (int64_t c = 0; c < n_chains; ++c) {
      for (int end = 0; end < 2; ++end) {
        const int j = end ? chain_lo[c] : chain_up[c];
        if (j < 0) continue;
        (end ? n_lo : n_up)[j] += 1;
        if (job_of_chain[c] != job_of_slot[j]) far[j] = 1;
      }
    }
    std::vector<int> rloc(n_slots, 0);
    std::vector<char> done_row(h->n_own - h->n_edge_dofs, 0);
    for (int64_t j = 0; j < n_slots; ++j) {
      const int pcn = slot_pchain[j];
      const bool ok = job_of_slot[j] >= 0 && !far[j] && slot_lam[j] < h->n_own &&
                      n_lo[j] == (pcn >= 0 ? 1 : 0) && (pcn < 0 || chain_lo[pcn] == j) &&
                      n_up[j] == slot_dc_off[j + 1] - slot_dc_off[j];
      rloc[j] = ok ? 1 : 0;
      if (ok) done_row[slot_lam[j] - h->n_edge_dofs] = 1;  // owned: slot_lam < n_own
    }
    std::vector<int> left;
    for (int64_t i = 0; i < (int64_t)done_row.size(); ++i)
      if (!done_row[i]) left.push_back((int)(h->n_edge_dofs + i));
    pa.slot_rloc = up(rloc.data(), n_slots);
    h->d_left = const_cast<int*>(up(left.empty() ? nullptr : left.data(), (int64_t)left.size()));
    pa.rpart = scratch(2 * (int64_t)n_jobs);
    h->dir_bb = scratch(1);
    pa.rres = h->tmp;
    pa.rhs_b = h->rhs;
    h->n_left = (int)left.size();
    h->fres_ok = pa.slot_rloc && h->d_left && pa.rpart && h->dir_bb && h->tmp;
    {  // k_dir_team_up's arrival counter (zero; its last workgroup resets it)
      unsigned* ty = nullptr;
      if (hipMalloc((void**)&ty, sizeof(unsigned)) == hipSuccess) {
        h->pc_bufs.push_back(ty);
        if (hipMemset(ty, 0, sizeof(unsigned)) != hipSuccess) ty = nullptr;
      }
      h->d_tsync = ty;
    }
    if (const char* e = std::getenv("NXHIP_DIR_FRES")) h->fres_ok = h->fres_ok && std::atoi(e) != 0;
    h->left_host = left;
    if (h->n_cut >= 0) {
      const int rc = build_left_cut(h);
      if (rc != NX_OK) return rc;
    }
    // the fused direct step (one rank, or a rank of several with its cut rows set): every
    // slot a job reads outside itself -- its root's parent, its chains' far ends -- is a top
    // slot (the down sweep takes it from the top values), and the rows no job forms get
    // their flux-end shares posted (chain order per row): the left rows and, with several
    // ranks, every cut bifurcation's row (owned or not: the K entries after the left rows,
    // which the publisher exchanges) instead of the cut rows among the left ones
    const bool xr_tables = h->nranks > 1 && h->n_cut >= 0;
    h->xr_ok = false;
    h->xr_nleft = 0;
    if (h->fres_ok && (h->nranks == 1 ? h->n_ghost == 0 : xr_tables)) {
      const int ts0 = top_lvl_off[0], ts1 = top_lvl_off[n_top_lvl];
      auto top = [&](int j) { return j >= ts0 && j < ts1; };
      bool ok = true;
      for (int64_t c = 0; c < n_chains && ok; ++c)
        for (int end = 0; end < 2; ++end) {
          const int j = end ? chain_lo[c] : chain_up[c];
          if (j >= 0 && job_of_slot[j] != job_of_chain[c] && !top(j)) ok = false;
        }
      for (int64_t j = 0; j < n_slots && ok; ++j) {
        const int p = slot_parent[j];
        if (job_of_slot[j] >= 0 && p >= 0 && job_of_slot[p] != job_of_slot[j] && !top(p)) ok = false;
      }
      const int K = xr_tables ? h->n_cut : 0;
      std::vector<int> dleft;  // the fused publisher's own rows: left rows that are not cut
      for (int r : left)
        if (!(xr_tables && h->lm_cut[r - h->n_edge_dofs] >= 0)) dleft.push_back(r);
      const int nl = (int)dleft.size();
      std::vector<int> row_of(h->n_own - h->n_edge_dofs, -1);
      for (int i = 0; i < nl; ++i) row_of[dleft[i] - h->n_edge_dofs] = i;
      if (xr_tables)  // owned cut rows: entry nl + k
        for (int64_t m = 0; m < (int64_t)row_of.size(); ++m)
          if (h->lm_cut[m] >= 0) row_of[m] = nl + h->lm_cut[m];
      std::vector<int> cut_of_row;  // a ghost junction's cut index by this rank's flux-end row
      if (xr_tables) {
        cut_of_row.assign(h->n_edge_dofs, -1);
        for (int k = 0; k < K; ++k)
          for (int e = h->gk_off_host[k]; e < h->gk_off_host[k + 1]; ++e)
            cut_of_row[h->gk_row_host[e]] = nl + k;
      }
      const int N2 = 2 * N + 1;
      // the post group of chain c's end (0 top, 1 bottom) at slot j, or -1
      auto row_at = [&](int64_t c, int end, int j) {
        if (j < 0) return -1;
        const int lam = slot_lam[j];
        if (lam < h->n_own) return row_of[lam - h->n_edge_dofs];
        if (!xr_tables) return -1;
        const int e = chain_edge[c], fl = chain_flip[c];  // the chain's end flux row
        const bool q0 = (end == 0) != (fl != 0);
        return cut_of_row[(int64_t)e * N2 + (q0 ? 0 : 2 * N)];
      };
      std::vector<int> off(nl + K + 1, 0), fill(nl + K, 0);
      std::vector<int> cpost(2 * std::max<int64_t>(n_chains, 1), -1);
      for (int64_t c = 0; c < n_chains; ++c)
        for (int end = 0; end < 2; ++end) {
          const int r = row_at(c, end, end ? chain_lo[c] : chain_up[c]);
          if (r >= 0) off[r + 1] += 1;
        }
      for (int i = 0; i < nl + K; ++i) off[i + 1] += off[i];
      for (int64_t c = 0; c < n_chains; ++c)
        for (int end = 0; end < 2; ++end) {
          const int r = row_at(c, end, end ? chain_lo[c] : chain_up[c]);
          if (r >= 0) cpost[2 * c + end] = off[r] + fill[r]++;
        }
      if (xr_tables) {  // every ghost junction end must have found its cut row
        for (int64_t c = 0; c < n_chains && ok; ++c)
          for (int end = 0; end < 2; ++end) {
            const int j = end ? chain_lo[c] : chain_up[c];
            if (j >= 0 && slot_lam[j] >= h->n_own && cpost[2 * c + end] < 0) ok = false;
          }
        h->xr_nleft = nl;
      }
      h->d_chain_post = const_cast<int*>(up(cpost.data(), (int64_t)cpost.size()));
      h->d_left_off = const_cast<int*>(up(off.data(), (int64_t)off.size()));
      h->d_post = scratch(std::max(1, off.back()));
      unsigned* sy = nullptr;
      if (hipMalloc((void**)&sy, 8 * sizeof(unsigned)) == hipSuccess) {
        h->pc_bufs.push_back(sy);
        if (hipMemset(sy, 0, 8 * sizeof(unsigned)) != hipSuccess) sy = nullptr;
      }
      h->d_dsync = sy;
      const bool tables = ok && h->d_chain_post && h->d_left_off && h->d_post && h->d_dsync;
      if (xr_tables)
        h->xr_ok = tables;  // (the exchange itself is checked per solve: xr_on)
      else
        h->dstep_ok = tables;
    }
  }
  pa.top_reg = 1;
  // the up sweep's one-wave level set-up (k_pc_up_lds): per eligible job (<= 64 slots, <=
  // kCapLvl levels, <= kWaveKids junction children per slot) each slot's level, children
  // (local slot) and their hanging-chain entries (offset from the job's first), packed
  pa.job_wave = nullptr;
  pa.slot_wave = nullptr;
  if (lds && n_jobs > 0) {
    std::vector<int> jw(n_jobs, 0), sw(3 * std::max<int64_t>(1, n_slots), 0);
    int n_wave = 0;
    for (int jb = 0; jb < n_jobs; ++jb) {
      const int lv0 = job_lvl_off[jb], lv1 = job_lvl_off[jb + 1];
      if (lv1 <= lv0) continue;
      const int js0 = lvl_slot_off[lv0], js1 = lvl_slot_off[lv1];
      if (js1 - js0 > 64 || lv1 - lv0 > kCapLvl) continue;
      const int dc0 = slot_dc_off[js0];
      bool ok = true;
      int kmax = 0;
      for (int lv = lv0; lv < lv1 && ok; ++lv)
        for (int j = lvl_slot_off[lv]; j < lvl_slot_off[lv + 1] && ok; ++j) {
          int nk = 0, cw[kWaveKids] = {0, 0, 0, 0};
          for (int i = slot_dc_off[j]; i < slot_dc_off[j + 1]; ++i) {
            if (dc_lo[i] < 0) continue;
            const int cl = dc_lo[i] - js0, off = i - dc0;
            if (nk >= kWaveKids || cl < 0 || cl >= 64 || off >= 1024) {
              ok = false;
              break;
            }
            cw[nk++] = cl | (off << 6);
          }
          kmax = std::max(kmax, nk);
          sw[3 * j] = (lv - lv0) | (nk << 8);
          sw[3 * j + 1] = cw[0] | (cw[1] << 16);
          sw[3 * j + 2] = cw[2] | (cw[3] << 16);
        }
      if (ok) {
        jw[jb] = kmax + 1;
        ++n_wave;
      }
    }
    if (n_wave > 0) {
      pa.job_wave = up(jw.data(), n_jobs);
      pa.slot_wave = up(sw.data(), (int64_t)sw.size());
    }
  }
  // the top part's register set-up (top_body): every slot's level, junction children (top
  // position) and their hanging-chain entries, when all have <= kWaveKids and fit
  pa.top_wave = nullptr;
  pa.top_sub = pa.top_lane = pa.top_sub_dep = nullptr;
  pa.top_sub_nup = 0;
  if (n_top_lvl > 0 && h->top_nt > 0 && h->top_nt <= kTopThreads) {
    const int ts0 = top_lvl_off[0], nt = h->top_nt, dc0 = slot_dc_off[ts0];
    std::vector<int> tw((size_t)(1 + kWaveKids) * nt, 0);
    bool ok = slot_dc_off[ts0 + nt] - dc0 < (1 << 19);
    for (int q = 0; q < n_top_lvl && ok; ++q)
      for (int j = top_lvl_off[q]; j < top_lvl_off[q + 1] && ok; ++j) {
        int nk = 0;
        int* w = tw.data() + (size_t)(1 + kWaveKids) * (j - ts0);
        for (int i = slot_dc_off[j]; i < slot_dc_off[j + 1]; ++i) {
          const int lo = dc_lo[i];
          if (!(lo >= ts0 && lo < ts0 + nt)) continue;  // a junction child in the top part
          if (nk >= kWaveKids || q > 0xff) {
            ok = false;
            break;
          }
          w[1 + nk++] = (lo - ts0) | ((i - dc0) << 12);
        }
        w[0] = q | (nk << 8);
      }
    if (ok) pa.top_wave = up(tw.data(), (int64_t)tw.size());
    // the same top part as wave subtrees (top_body): maximal subtrees of <= 64 slots, one per
    // wave, BFS lanes; the slots above them swept level by level (NXHIP_TOP_SUB=0: all levels)
    const char* es = std::getenv("NXHIP_TOP_SUB");
    if (ok && (es == nullptr || std::atoi(es) != 0)) {
      constexpr int K1 = 1 + kWaveKids, K2 = 2 + kWaveKids, NW = kTopThreads / 64;
      std::vector<int> lvl(nt, 0), size(nt, 1), par(nt, -1);
      for (int q = 0; q < n_top_lvl; ++q)
        for (int j = top_lvl_off[q]; j < top_lvl_off[q + 1]; ++j) lvl[j - ts0] = q;
      for (int q = n_top_lvl - 1; q >= 0; --q)  // subtree sizes, deepest level first
        for (int j = top_lvl_off[q]; j < top_lvl_off[q + 1]; ++j) {
          const int* w = tw.data() + (size_t)K1 * (j - ts0);
          for (int k = 0; k < ((w[0] >> 8) & 0xff); ++k) {
            const int c = w[1 + k] & 0xfff;
            size[j - ts0] += size[c];
            par[c] = j - ts0;
          }
        }
      std::vector<int> ts(K1 * (size_t)nt, 0), tl(K2 * (size_t)kTopThreads, 0), tdep(NW, 0);
      for (int t = 0; t < kTopThreads; ++t) tl[(size_t)K2 * t] = -1;
      int nup = 0;
      bool sok = true;
      std::vector<int> roots;  // the maximal subtrees' roots
      for (int j = 0; j < nt; ++j) {
        if (size[j] > 64) {  // an upper slot: the level sweeps
          const int* w = tw.data() + (size_t)K1 * j;
          int* o = ts.data() + (size_t)K1 * j;
          o[0] = (int)(0x80000000u | (unsigned)w[0]);
          for (int k = 0; k < kWaveKids; ++k) o[1 + k] = w[1 + k];
          nup = std::max(nup, lvl[j] + 1);
        } else if (par[j] < 0 || size[par[j]] > 64) {
          roots.push_back(j);
        }
      }
      // packed into the waves first-fit by decreasing size: lanes of different subtrees never
      // exchange values, so a wave sweeps all of its subtrees at once
      std::stable_sort(roots.begin(), roots.end(), [&](int a, int b) { return size[a] > size[b]; });
      std::vector<int> fill(NW, 0);
      int nsub = 0;
      for (int j : roots) {
        int wv = 0;
        while (wv < NW && fill[wv] + size[j] > 64) ++wv;
        if (wv == NW) {
          sok = false;
          break;
        }
        const int base = fill[wv];
        fill[wv] += size[j];
        nsub = std::max(nsub, wv + 1);
        std::vector<int> bfs{j}, lane_of(nt, -1), dep{0};  // this subtree, BFS order
        lane_of[j] = base;
        for (size_t i = 0; i < bfs.size(); ++i) {
          const int* w = tw.data() + (size_t)K1 * bfs[i];
          for (int k = 0; k < ((w[0] >> 8) & 0xff); ++k) {
            const int c = w[1 + k] & 0xfff;
            lane_of[c] = base + (int)bfs.size();
            bfs.push_back(c);
            dep.push_back(dep[i] + 1);
          }
        }
        int md = 0;
        for (size_t i = 0; i < bfs.size(); ++i) {
          const int m = bfs[i];
          const int* w = tw.data() + (size_t)K1 * m;
          const int nk = (w[0] >> 8) & 0xff;
          const int ln = base + (int)i;
          int* o = tl.data() + (size_t)K2 * (wv * 64 + ln);
          o[0] = m;
          const int pl = dep[i] > 0 ? lane_of[par[m]] : 0;
          o[1] = ln | (dep[i] << 6) | (nk << 14) | (pl << 18);
          for (int k = 0; k < nk; ++k) o[2 + k] = lane_of[w[1 + k] & 0xfff] | ((w[1 + k] >> 12) << 12);
          md = std::max(md, dep[i]);
        }
        if (md > 0xff) sok = false;
        tdep[wv] = std::max(tdep[wv], md + 1);
      }
      if (sok && nsub > 0) {
        pa.top_sub = up(ts.data(), (int64_t)ts.size());
        pa.top_lane = up(tl.data(), (int64_t)tl.size());
        pa.top_sub_dep = up(tdep.data(), NW);
        pa.top_sub_nup = nup;
      }
    }
  }
  // k_dir_step's job headers, stash strides, dynamic LDS and chain records (round 4)
  h->d_job_hdr = nullptr;
  h->d_crec = nullptr;
  h->d_ci = nullptr;
  if (h->dstep_ok || h->xr_ok) {
    std::vector<int> hdr((size_t)kJobHdr * n_jobs, 0);
    int mlv = 1, mns = 0, mnd = 0, mch = 0;
    for (int jb = 0; jb < n_jobs; ++jb) {
      const int lv0 = job_lvl_off[jb], lv1 = job_lvl_off[jb + 1];
      const int js0 = lv1 > lv0 ? lvl_slot_off[lv0] : 0, js1 = lv1 > lv0 ? lvl_slot_off[lv1] : 0;
      int* r = hdr.data() + (size_t)kJobHdr * jb;
      r[0] = job_chain_off[jb];
      r[1] = job_chain_off[jb + 1];
      r[2] = lv0;
      r[3] = lv1;
      r[4] = js0;
      r[5] = js1;
      r[6] = slot_dc_off[js0];
      r[7] = slot_dc_off[js1];
      r[8] = 0;
      r[9] = lv1 > lv0 ? lvl_slot_off[lv0 + 1] : 0;
      mlv = std::max(mlv, lv1 - lv0 + 1);
      mns = std::max(mns, js1 - js0);
      mnd = std::max(mnd, r[7] - r[6]);
      mch = std::max(mch, r[1] - r[0]);
    }
    if (pa.job_wave) {  // (the one-wave set-up of the up sweep, when the job has it)
      std::vector<int> jw(n_jobs, 0);
      HIPCALL(hipMemcpy(jw.data(), pa.job_wave, sizeof(int) * n_jobs, hipMemcpyDeviceToHost));
      for (int jb = 0; jb < n_jobs; ++jb) hdr[(size_t)kJobHdr * jb + 8] = jw[jb];
    }
    const int W = variant_w(N <= 16 ? 5 : N <= 24 ? 10 : N <= 32 ? 7 : variant);  // (dstep's)
    h->dstep_multi = mch > kPcThreads / W;
    const int nt = h->top_nt, cdc = std::max(1, pa.top_ndc), ct = nt + 1;
    const int top_ints = 3 * ct + 1 + cdc + n_top_lvl + 1;
    const int top_dbl = 6 * ct + 3 * cdc + (top_ints + 1) / 2 + 2;
    // (several ranks: xr_top_back's per-slot T and coarse index after the top part)
    const int xr_dbl = h->nranks > 1 ? 2 * (nt + 1) + 4 : 0;
    h->dstep_main = std::max({kDirLdsPhase1, kDirLdsPhase2, top_dbl + xr_dbl});
    h->dstep_top = nt + (nt & 1);
    h->dstep_lds = 8 * (size_t)(kStashDbl + h->dstep_main + h->dstep_top + kDirLdsSupSlots);
    {  // phase 2 by superposition: its park (2 CPL + 1 doubles per thread), when it fits (with
       // the exchange kernels' static LDS on several ranks)
      const int dv = N <= 16 ? 5 : N <= 24 ? 10 : N <= 32 ? 7 : variant;
      const size_t park = 8 * (size_t)(2 * variant_cpl(dv) + 1) * kPcThreads;
      // (several ranks: the exchange kernels' static LDS comes on top; the rank count is set
      // before the preconditioner -- nx_set_halo refuses to run after it)
      const size_t cap = h->nranks > 1 ? std::min((size_t)kDirLdsMax, 160 * 1024 - xr_static_lds(dv))
                                       : (size_t)kDirLdsMax;
      h->dstep_park = h->dstep_lds + park <= cap;
      if (h->dstep_park) h->dstep_lds += park;
      const size_t recs = 8 * ((size_t)kRecLds * (kPcThreads / variant_w(dv)) +
                               2 * (size_t)variant_cpl(dv) * kPcThreads);
      h->dstep_rec = h->dstep_park && h->dstep_lds + recs <= cap;
      if (h->dstep_rec) h->dstep_lds += recs;
    }
    const bool fits = mlv <= kStLv && mns <= kStNs && mnd <= kStNd && kPcThreads / W <= kStNc;
    h->d_job_hdr = const_cast<int*>(up(hdr.data(), (int64_t)hdr.size()));
    h->d_crec = scratch(10 * std::max<int64_t>(n_chains, 1));
    h->d_ci = const_cast<int*>(up(nullptr, 4 * std::max<int64_t>(n_chains, 1)));
    const bool hdr_ok = h->d_job_hdr && h->d_crec && h->d_ci && fits;
    // (N > 256, variants <64, 8> / <64, 16>: the lane state spills thousands of VGPRs -- the
    // separate launches run those; no fused instantiation)
    h->dstep_ok = h->dstep_ok && hdr_ok && h->dstep_lds <= (size_t)kDirLdsMax &&
                  (N <= 32 || (variant != 8 && variant != 9));
    // (several ranks: the coarse exchange's static LDS comes on top; checked at launch)
    h->xr_ok = h->xr_ok && hdr_ok;
  }
  h->pc_lds = lds;
  h->pa = pa;
  h->pc_jobs = n_jobs;
  h->pc_variant = variant;
  h->dstep_variant = N <= 16 ? 5 : N <= 24 ? 10 : N <= 32 ? 7 : variant;
  if (h->d_crec) CHECK(chain_rec_refresh(h));
  h->pc_slots = n_slots;
  h->pc_ndc = n_slots > 0 ? slot_dc_off[n_slots] : 0;
  h->pc = true;
  return NX_OK;
}

NX_API int nx_set_pc_dense(nx_network_t* h, int32_t enable, int32_t n_jobs,
                           const int32_t* job_tslot_off, const int32_t* job_tslot,
                           const int32_t* job_need_off, const int32_t* job_need,
                           const int32_t* top_uoff, const int32_t* slot_uy,
                           const int32_t* chain_uit, const int32_t* chain_uib,
                           const int32_t* job_root_u, const int32_t* job_root_dc) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (!h->pc) return fail(NX_ERR_STATE, "nx_set_preconditioner(enable=1) must come first");
  h->sched_checked = false;
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  CHECK(drop_handle_graphs(h));
  h->pa.dense = 0;
  if (!enable) return NX_OK;
  if (n_jobs != h->pc_jobs) return fail(NX_ERR_ARG, "n_jobs differs from the preconditioner's");
  std::vector<int> top_off(h->pa.n_top_lvl + 1);
  HIPCALL(hipMemcpy(top_off.data(), h->pa.top_lvl_off, sizeof(int) * top_off.size(),
                    hipMemcpyDeviceToHost));
  const int ts0 = top_off[0], nt = top_off.back() - top_off[0];
  if (job_tslot_off[0] != 0 || job_need_off[0] != 0 || job_tslot_off[n_jobs] != nt)
    return fail(NX_ERR_ARG, "job_tslot must cover the top slots once");
  bool fits = true;  // a job reading more than kMaxNeed top values keeps the top kernel
  for (int j = 0; j < n_jobs; ++j)
    if (job_need_off[j + 1] - job_need_off[j] > kMaxNeed) fits = false;
  for (int i = 0; i < nt; ++i)
    if (job_tslot[i] < ts0 || job_tslot[i] >= ts0 + nt) return fail(NX_ERR_ARG, "job_tslot out of range");
  for (int i = 0; i < job_need_off[n_jobs]; ++i)
    if (job_need[i] < ts0 || job_need[i] >= ts0 + nt) return fail(NX_ERR_ARG, "job_need out of range");
  const int n_u = top_uoff[nt];
  if (top_uoff[0] != 0 || n_u < nt) return fail(NX_ERR_ARG, "bad top_uoff");
  for (int i = 0; i < nt; ++i)
    if (slot_uy[i] < 0 || slot_uy[i] >= n_u) return fail(NX_ERR_ARG, "slot_uy out of range");
  for (int64_t c = 0; c < h->E; ++c)
    if (chain_uit[c] >= n_u || chain_uib[c] >= n_u) return fail(NX_ERR_ARG, "chain_u* out of range");
  for (int j = 0; j < n_jobs; ++j)
    if (job_root_u[j] >= n_u || job_root_dc[j] >= h->pc_ndc ||
        (job_root_u[j] >= 0 && job_root_dc[j] < 0))
      return fail(NX_ERR_ARG, "job_root_u / job_root_dc out of range");
  // dense mode: single rank, LDS kernels, a top part that fits
  if (!fits || !h->pc_lds || nt < 1 || nt > kCapT || n_jobs < 1) return NX_OK;
  auto up = [&](const int32_t* src, int64_t n) -> const int* {
    int* d = nullptr;
    if (n <= 0) n = 1;
    if (hipMalloc((void**)&d, sizeof(int) * n) != hipSuccess) return nullptr;
    h->pc_bufs.push_back(d);
    if (hipMemcpy(d, src, sizeof(int) * n, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return d;
  };
  PcArgs& pa = h->pa;
  pa.job_tslot_off = up(job_tslot_off, n_jobs + 1);
  pa.job_tslot = up(job_tslot, nt);
  pa.job_need_off = up(job_need_off, n_jobs + 1);
  pa.job_need = up(job_need, std::max(1, job_need_off[n_jobs]));
  pa.top_uoff = up(top_uoff, nt + 1);
  pa.slot_uy = up(slot_uy, nt);
  pa.chain_uit = up(chain_uit, h->E);
  pa.chain_uib = up(chain_uib, h->E);
  pa.job_root_u = up(job_root_u, n_jobs);
  pa.job_root_dc = up(job_root_dc, n_jobs);
  double* ub = nullptr;
  HIPCALL(hipMalloc((void**)&ub, sizeof(double) * n_u));
  HIPCALL(hipMemset(ub, 0, sizeof(double) * n_u));
  h->pc_bufs.push_back(ub);
  pa.u = ub;
  double* G = nullptr;
  HIPCALL(hipMalloc((void**)&G, sizeof(double) * (size_t)nt * nt));
  h->pc_bufs.push_back(G);
  pa.G = G;
  pa.KJ = nullptr;
  if (h->nranks > 1) {  // several ranks: top trees rooted at coarse junctions (Dirichlet)
    double *kj = nullptr, *w = nullptr, *at = nullptr;
    int* rc = nullptr;
    HIPCALL(hipMalloc((void**)&kj, sizeof(double) * (size_t)nt * nt));
    h->pc_bufs.push_back(kj);
    HIPCALL(hipMalloc((void**)&w, sizeof(double) * nt));
    h->pc_bufs.push_back(w);
    HIPCALL(hipMalloc((void**)&at, sizeof(double) * nt));
    h->pc_bufs.push_back(at);
    HIPCALL(hipMalloc((void**)&rc, sizeof(int) * nt));
    h->pc_bufs.push_back(rc);
    pa.KJ = kj;
    pa.top_w = w;
    pa.atop = at;
    pa.top_rootc = rc;
  }
  if (!pa.job_tslot_off || !pa.job_tslot || !pa.job_need_off || !pa.job_need || !pa.top_uoff ||
      !pa.slot_uy || !pa.chain_uit || !pa.chain_uib || !pa.job_root_u || !pa.job_root_dc)
    return fail(NX_ERR_HIP, "dense top upload failed");
  pa.n_top = nt;
  pa.dense = 1;
  return NX_OK;
}

namespace {
void free_cycles(nx_network* h) {
  for (void* p : {(void*)h->d_cyc_rows, (void*)h->cyc_z, (void*)h->cyc_cinv, (void*)h->cyc_cap,
                  (void*)h->cyc_prev, (void*)h->cyc_w, (void*)h->d_cyc_qloc, (void*)h->d_cyc_lcol,
                  (void*)h->cyc_u, (void*)h->cyc_gj})
    if (p) (void)hipFree(p);
  h->cyc_gj = nullptr;
  h->d_cyc_rows = h->d_cyc_qloc = h->d_cyc_lcol = nullptr;
  h->cyc_z = h->cyc_cinv = h->cyc_cap = h->cyc_prev = h->cyc_w = h->cyc_u = nullptr;
  h->cyc_team = false;
  h->n_cyc = 0;
  h->cyc_version = -1;
}
}  // namespace

NX_API int nx_set_cycles(nx_network_t* h, int32_t n, const int32_t* rows) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (n < 0 || (n > 0 && !rows)) return fail(NX_ERR_ARG, "n >= 0 row pairs");
  if (n > 0 && !h->pc) return fail(NX_ERR_STATE, "nx_set_preconditioner(enable=1) must come first");
  if (n > 0 && (h->nranks > 1 || proc_rank(h) || h->group || h->n_ghost > 0))
    return fail(NX_ERR_STATE, "the cycle correction is one rank's");
  if (n > kMaxCyc) return fail(NX_ERR_ARG, "more cycle chains than kMaxCyc (the solve runs MINRES)");
  for (int64_t i = 0; i < 2 * (int64_t)n; ++i)
    if (rows[i] < 0 || rows[i] >= h->n_own) return fail(NX_ERR_ARG, "cycle row out of range");
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  CHECK(drop_handle_graphs(h));
  free_cycles(h);
  if (n == 0) return NX_OK;
  const int m = 2 * n;
  HIPCALL(hipMalloc((void**)&h->d_cyc_rows, sizeof(int) * m));
  HIPCALL(hipMalloc((void**)&h->cyc_z, sizeof(double) * m * h->n_col));
  HIPCALL(hipMalloc((void**)&h->cyc_cinv, sizeof(double) * m * m));
  HIPCALL(hipMalloc((void**)&h->cyc_cap, sizeof(double) * (m * m + n)));
  HIPCALL(hipMalloc((void**)&h->cyc_prev, sizeof(double) * m));
  HIPCALL(hipMalloc((void**)&h->cyc_w, sizeof(double) * m));
  HIPCALL(hipMemcpy(h->d_cyc_rows, rows, sizeof(int) * m, hipMemcpyHostToDevice));
  h->n_cyc = n;
  // the residual check of the corrected x is the CSR's (the sweeps' fused one is A_g's), so
  // neither the fused residual nor the fused step run
  h->fres_ok = false;
  h->dstep_ok = false;
  return NX_OK;
}

// Several ranks, a graph with cycles: this rank's share of the Woodbury correction. K: the
// cycle chains of all ranks (one global order, the same on every rank); own[2K]: per column
// of U (flux end, multiplier of pair k at 2k, 2k + 1) this rank's row or -1; qloc[K] /
// lcol[K]: when pair k's chain is this rank's, its flux end row and the multiplier's column
// in this rank's numbering (a ghost column when another rank owns the row), else -1.
NX_API int nx_set_cycles_team(nx_network_t* h, int32_t K, const int32_t* own,
                              const int32_t* qloc, const int32_t* lcol) {
  CHECK(flush_assembly(h));
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (K < 0 || (K > 0 && (!own || !qloc || !lcol))) return fail(NX_ERR_ARG, "K >= 0 pairs");
  if (K > 0 && !h->pc) return fail(NX_ERR_STATE, "nx_set_preconditioner(enable=1) must come first");
  if (K > 0 && h->nranks < 2) return fail(NX_ERR_STATE, "one rank: nx_set_cycles");
  if (K > kMaxCyc) return fail(NX_ERR_ARG, "more cycle chains than kMaxCyc (the solve runs MINRES)");
  for (int64_t i = 0; i < 2 * (int64_t)K; ++i)
    if (own[i] < -1 || own[i] >= h->n_own) return fail(NX_ERR_ARG, "cycle row out of range");
  for (int k = 0; k < K; ++k)
    if (qloc[k] < -1 || qloc[k] >= h->n_edge_dofs || lcol[k] < -1 || lcol[k] >= h->n_col ||
        (qloc[k] >= 0) != (lcol[k] >= 0))
      return fail(NX_ERR_ARG, "cycle chain row / column out of range");
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  CHECK(drop_handle_graphs(h));
  free_cycles(h);
  h->sched_checked = false;
  if (K == 0) return NX_OK;
  const int m = 2 * K;
  HIPCALL(hipMalloc((void**)&h->d_cyc_rows, sizeof(int) * m));
  HIPCALL(hipMalloc((void**)&h->d_cyc_qloc, sizeof(int) * K));
  HIPCALL(hipMalloc((void**)&h->d_cyc_lcol, sizeof(int) * K));
  HIPCALL(hipMalloc((void**)&h->cyc_z, sizeof(double) * m * h->n_col));
  HIPCALL(hipMalloc((void**)&h->cyc_cinv, sizeof(double) * m * m));
  HIPCALL(hipMalloc((void**)&h->cyc_cap, sizeof(double) * (m * m + K)));
  HIPCALL(hipMalloc((void**)&h->cyc_prev, sizeof(double) * m));
  HIPCALL(hipMalloc((void**)&h->cyc_w, sizeof(double) * m));
  HIPCALL(hipMalloc((void**)&h->cyc_u, sizeof(double) * m));
  HIPCALL(hipMemcpy(h->d_cyc_rows, own, sizeof(int) * m, hipMemcpyHostToDevice));
  HIPCALL(hipMemcpy(h->d_cyc_qloc, qloc, sizeof(int) * K, hipMemcpyHostToDevice));
  HIPCALL(hipMemcpy(h->d_cyc_lcol, lcol, sizeof(int) * K, hipMemcpyHostToDevice));
  h->n_cyc = K;
  h->cyc_team = true;
  return NX_OK;
}

NX_API int nx_set_cell_mass(nx_network_t* h, double ratio, double mo_div) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (!h->pc || !h->pa.Tlu) return fail(NX_ERR_STATE, "nx_set_preconditioner(enable=1) must come first");
  if (h->fe) return fail(NX_ERR_STATE, "a P1/DG0 handle's preconditioner");
  if (!(std::fabs(ratio) > 1.0) || !std::isfinite(mo_div) || mo_div == 0.0)
    return fail(NX_ERR_ARG, "|ratio| must exceed 1 (a diagonally dominant T) and mo_div != 0");
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  CHECK(drop_handle_graphs(h));
  const std::vector<double> ti = mass_lu(h->N, ratio);
  HIPCALL(hipMemcpy(const_cast<double*>(h->pa.Tlu), ti.data(), sizeof(double) * ti.size(),
                    hipMemcpyHostToDevice));
  h->pa.mo_div = mo_div;
  h->cond_mass = !(ratio == 2.0 && mo_div == 3.0);
  if (h->cond_mass) {  // the fused residual and the fused step regenerate P1's masses
    h->fres_ok = false;
    h->dstep_ok = false;
  }
  h->sched_checked = false;
  return NX_OK;
}

// Several ranks, continuous pressure: this rank's part of the node-condensed direct solve,
// given before nx_fe_set_cp (whose eb / nown then list this rank's n_own_edges edges and whose
// node tables name global edges). gid: the global edge of each of them; nrowx (2 per node):
// the local rows of the node rows this rank owns, -1 elsewhere.
NX_API int nx_fe_cp_ranks(nx_network_t* h, int64_t n_own_edges, int64_t n_edges_global,
                          const int32_t* gid, int64_t n_nodes, const int32_t* nrowx) {
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (!h->fe) return fail(NX_ERR_STATE, "a general-degree handle (nx_create_fe)");
  if (n_own_edges < 0 || n_own_edges > h->E || n_edges_global < n_own_edges || n_nodes < 1 ||
      (n_own_edges > 0 && !gid) || !nrowx)
    return fail(NX_ERR_ARG, "bad rank tables");
  for (int64_t e = 0; e < n_own_edges; ++e)
    if (gid[e] < 0 || gid[e] >= n_edges_global) return fail(NX_ERR_ARG, "gid out of range");
  for (int64_t i = 0; i < 2 * n_nodes; ++i)
    if (nrowx[i] < -1 || nrowx[i] >= h->n_own) return fail(NX_ERR_ARG, "nrowx out of range");
  h->cp_Eown = n_own_edges;
  h->cp_Eg = n_edges_global;
  h->cp_gid_host.assign(gid ? gid : nullptr, gid ? gid + n_own_edges : nullptr);
  h->cp_nrowx_host.assign(nrowx, nrowx + 2 * n_nodes);
  return NX_OK;
}

// Continuous pressure (k > m >= 1), a forest: attach the node-condensed direct solve (see
// include/nxhip.h); k = 0 detaches it.
NX_API int nx_fe_set_cp(nx_network_t* h, int32_t k, int32_t m, int32_t nI, const double* cst,
                        const int32_t* tI, int64_t n_nodes, const int32_t* nrow, const int32_t* eb,
                        int32_t n_lev, const int32_t* lev_off, const int32_t* order,
                        const int32_t* inc_off, const int32_t* inc, const int32_t* parent,
                        const int32_t* child_off, const int32_t* child, const int32_t* nown) {
  CHECK(flush_assembly(h));
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (!h->fe) return fail(NX_ERR_STATE, "a general-degree handle (nx_create_fe)");
  // several ranks: nx_fe_cp_ranks first (this rank's edges and the global edge count)
  const bool ranks = !h->cp_gid_host.empty() || h->cp_Eg > 0;
  if (k != 0 && (h->nranks > 1 || h->n_ghost > 0) && !ranks)
    return fail(NX_ERR_STATE, "several ranks: nx_fe_cp_ranks before nx_fe_set_cp");
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  for (double** p : {&h->cp_cst, &h->cp_fac, &h->cp_se, &h->cp_xn, &h->cp_Pinv, &h->cp_hv,
                     &h->cp_ctr}) {
    if (*p) HIPCALL(hipFree(*p));
    *p = nullptr;
  }
  for (int** p : {&h->cp_tI, &h->cp_eb, &h->cp_nrow, &h->cp_lev_off, &h->cp_order, &h->cp_inc_off,
                  &h->cp_inc, &h->cp_parent, &h->cp_child_off, &h->cp_child, &h->cp_nown,
                  &h->cp_gid, &h->cp_nrowx, &h->cp_rec, &h->cp_rng}) {
    if (*p) HIPCALL(hipFree(*p));
    *p = nullptr;
  }
  h->cp_runs.clear();
  h->fe_cp = false;
  if (k == 0) {
    h->cp_Eown = h->cp_Eg = 0;
    h->cp_gid_host.clear();
    h->cp_nrowx_host.clear();
    return NX_OK;
  }
  // E: the edges the edge kernels run (eb rows, nown); Es: the edges the node tables name
  const int64_t n = n_nodes, E = ranks ? h->cp_Eown : h->E, Es = ranks ? h->cp_Eg : h->E;
  if (!(m >= 1 && k > m) || nI != (k - 1) + (m - 1) || n < 1 || n_lev < 1 || !cst || !nrow ||
      !eb || !lev_off || !order || !inc_off || !inc || !parent || !child_off || !nown ||
      (nI > 0 && !tI))
    return fail(NX_ERR_ARG, "bad continuous-pressure tables");
  if (!ranks && h->n_own < E * (int64_t)(k * h->N + 1 + m * h->N - 1) + n)
    return fail(NX_ERR_ARG, "row counts do not match a (k, m) layout");
  if (ranks && (h->n_own < E * (int64_t)(k * h->N + 1 + m * h->N - 1) ||
                (int64_t)h->cp_nrowx_host.size() != 2 * n))
    return fail(NX_ERR_ARG, "several ranks: rows / node rows do not match the tables");
  // one rank: nrow are rows; several: indices of the summed node rhs (2 per node)
  const int64_t nlim = ranks ? 2 * n : h->n_own;
  for (int64_t i = 0; i < n; ++i)
    if (nrow[2 * i] < 0 || nrow[2 * i] >= nlim || nrow[2 * i + 1] < -1 || nrow[2 * i + 1] >= nlim ||
        parent[3 * i] < -1 || parent[3 * i] >= n || parent[3 * i + 1] < -1 || parent[3 * i + 1] >= Es ||
        nown[i] < (ranks ? -1 : 0) || nown[i] >= E)
      return fail(NX_ERR_ARG, "continuous pressure: node tables out of range");
  for (int64_t e = 0; e < E; ++e)
    if (eb[4 * e] < 0 || eb[4 * e] >= n || eb[4 * e + 1] < 0 || eb[4 * e + 1] >= n ||
        std::abs(eb[4 * e + 2]) > 1 || std::abs(eb[4 * e + 3]) > 1)
      return fail(NX_ERR_ARG, "continuous pressure: edge tables out of range");
  if (lev_off[0] != 0 || lev_off[n_lev] != n || inc_off[0] != 0 || child_off[0] != 0)
    return fail(NX_ERR_ARG, "continuous pressure: offsets");
  // (the host's record builder and the kernels index through these: monotone, and within
  // what the tables can hold -- an edge has two ends, a node at most one parent)
  for (int64_t i = 0; i < n_lev; ++i)
    if (lev_off[i + 1] < lev_off[i]) return fail(NX_ERR_ARG, "continuous pressure: level offsets");
  for (int64_t i = 0; i < n; ++i)
    if (inc_off[i + 1] < inc_off[i] || child_off[i + 1] < child_off[i] || parent[3 * i + 2] < -1 ||
        parent[3 * i + 2] > 1)
      return fail(NX_ERR_ARG, "continuous pressure: offsets / parent end");
  if (inc_off[n] > 2 * Es || child_off[n] > n)
    return fail(NX_ERR_ARG, "continuous pressure: more incidences or children than the graph has");
  for (int64_t i = 0; i < n; ++i)
    if (order[i] < 0 || order[i] >= n) return fail(NX_ERR_ARG, "continuous pressure: order");
  for (int64_t j = 0; j < inc_off[n]; ++j)
    if (inc[2 * j] < 0 || inc[2 * j] >= Es || inc[2 * j + 1] < 0 || inc[2 * j + 1] > 1)
      return fail(NX_ERR_ARG, "continuous pressure: incidence");
  for (int64_t j = 0; j < child_off[n]; ++j)
    if (child[j] < 0 || child[j] >= n) return fail(NX_ERR_ARG, "continuous pressure: children");
  const int64_t ncst = 16 + 8 * (int64_t)nI + (int64_t)nI * nI;
  CHECK(upload(&h->cp_cst, cst, ncst, h->stream));
  if (nI > 0) CHECK(upload(&h->cp_tI, tI, nI, h->stream));
  CHECK(upload(&h->cp_nrow, nrow, 2 * n, h->stream));
  CHECK(upload(&h->cp_eb, eb, 4 * E, h->stream));
  CHECK(upload(&h->cp_lev_off, lev_off, (int64_t)n_lev + 1, h->stream));
  CHECK(upload(&h->cp_order, order, n, h->stream));
  CHECK(upload(&h->cp_inc_off, inc_off, n + 1, h->stream));
  CHECK(upload(&h->cp_inc, inc, std::max<int64_t>(1, 2 * (int64_t)inc_off[n]), h->stream));
  CHECK(upload(&h->cp_parent, parent, 3 * n, h->stream));
  CHECK(upload(&h->cp_child_off, child_off, n + 1, h->stream));
  if (child_off[n] > 0) CHECK(upload(&h->cp_child, child, child_off[n], h->stream));
  CHECK(upload(&h->cp_nown, nown, n, h->stream));
  {  // the node records in level order (CpTree::rec; the same sums in the same order)
    // the levels from the first wider than kCpChunk nodes to the deepest (one run): their
    // nodes re-ordered inside each level by their ancestor at the run's first level (stable),
    // so a range of those ancestors owns one range per level -- a chunk, one workgroup's
    // subtrees of at most kCpChunk nodes per level (cp_nodes_launch; one CU moves a level's
    // few hundred bytes per node at a few tens of GB/s, so the chunks stay small). Within a
    // level the nodes are independent: the order changes no sum.
    std::vector<int> ord(order, order + n), lvl_of(n, 0), anc(n, -1);
    for (int L = 0; L < n_lev; ++L)
      for (int i = lev_off[L]; i < lev_off[L + 1]; ++i) lvl_of[order[i]] = L;
    std::vector<int> rng;
    int Lc = 0;
    while (Lc < n_lev && lev_off[Lc + 1] - lev_off[Lc] <= kCpChunk) ++Lc;
    for (int L = Lc; L < n_lev;) {
      const int L1 = n_lev;
      bool ok = L1 - L <= kCpPipeLv;
      for (int i = lev_off[L]; i < lev_off[L + 1]; ++i) anc[ord[i]] = i - lev_off[L];
      for (int Q = L + 1; Q < L1 && ok; ++Q) {
        for (int i = lev_off[Q]; i < lev_off[Q + 1]; ++i) {
          const int nd = ord[i], pn = parent[3 * nd];
          if (pn < 0 || lvl_of[pn] != Q - 1) {
            ok = false;  // (a BFS forest: the parent is one level up)
            break;
          }
          anc[nd] = anc[pn];
        }
        if (ok)
          std::stable_sort(ord.begin() + lev_off[Q], ord.begin() + lev_off[Q + 1],
                           [&](int x, int y) { return anc[x] < anc[y]; });
      }
      if (ok) {  // chunks of ancestors, at most 1024 nodes per level
        const int na = lev_off[L + 1] - lev_off[L], nq = L1 - L;
        std::vector<std::vector<int>> cnt(nq, std::vector<int>(na, 0));
        for (int Q = L; Q < L1; ++Q)
          for (int i = lev_off[Q]; i < lev_off[Q + 1]; ++i) cnt[Q - L][anc[ord[i]]] += 1;
        std::vector<int> start(nq), cur(nq, 0);
        for (int Q = 0; Q < nq; ++Q) start[Q] = lev_off[L + Q];
        nx_network::CpRun run{L, L1, 0, (int)rng.size()};
        int a0 = 0;
        while (a0 < na && ok) {
          int a1 = a0;
          std::vector<int> sum(nq, 0);
          while (a1 < na) {
            bool fits = true;
            for (int Q = 0; Q < nq; ++Q) fits = fits && sum[Q] + cnt[Q][a1] <= kCpChunk;
            if (!fits) break;
            for (int Q = 0; Q < nq; ++Q) sum[Q] += cnt[Q][a1];
            ++a1;
          }
          if (a1 == a0) {
            ok = false;  // (one ancestor with more than kCpChunk descendants on a level)
            break;
          }
          for (int Q = 0; Q < nq; ++Q) {
            rng.push_back(start[Q] + cur[Q]);
            cur[Q] += sum[Q];
            rng.push_back(start[Q] + cur[Q]);
          }
          run.nch += 1;
          a0 = a1;
        }
        if (ok)
          h->cp_runs.push_back(run);
        else
          rng.resize(run.off);
      }
      if (!ok)  // (this run stays level by level: its original order)
        for (int Q = L; Q < L1; ++Q)
          for (int i = lev_off[Q]; i < lev_off[Q + 1]; ++i) ord[i] = order[i];
      L = L1;
    }
    std::vector<int> rec((size_t)n * kCpRecPad, 0);
    h->cp_lev_full.assign(n_lev, 1);
    for (int L = 0; L < n_lev; ++L)
      for (int i = lev_off[L]; i < lev_off[L + 1]; ++i) {
        const int nd = order[i];
        if (inc_off[nd + 1] - inc_off[nd] > kCpRecInc || child_off[nd + 1] - child_off[nd] > kCpRecCh)
          h->cp_lev_full[L] = 0;
      }
    for (size_t q = 0; q < h->cp_runs.size();)  // (a run with an overflowing record: by levels)
      if (std::any_of(h->cp_lev_full.begin() + h->cp_runs[q].L0,
                      h->cp_lev_full.begin() + h->cp_runs[q].L1, [](char f) { return !f; }))
        h->cp_runs.erase(h->cp_runs.begin() + q);
      else
        ++q;
    for (int64_t i = 0; i < n; ++i) {
      int* r = rec.data() + i * kCpRecPad;
      const int nd = ord[i];
      r[0] = nd;
      r[1] = nrow[2 * nd];
      r[2] = nrow[2 * nd + 1];
      const int ni = inc_off[nd + 1] - inc_off[nd], nc = child_off[nd + 1] - child_off[nd];
      r[3] = ni <= kCpRecInc ? ni : -1;
      for (int j = 0; j < ni && ni <= kCpRecInc; ++j) {
        r[4 + 2 * j] = inc[2 * (inc_off[nd] + j)];
        r[5 + 2 * j] = inc[2 * (inc_off[nd] + j) + 1];
      }
      constexpr int kc = kCpRecC;
      r[kc] = nc <= kCpRecCh ? nc : -1;
      for (int j = 0; j < nc && nc <= kCpRecCh; ++j) {
        const int c = child[child_off[nd] + j];
        r[kc + 1 + 3 * j] = c;
        r[kc + 2 + 3 * j] = parent[3 * c + 1];
        r[kc + 3 + 3 * j] = parent[3 * c + 2];
      }
      r[kCpRecP] = parent[3 * nd];
      r[kCpRecP + 1] = parent[3 * nd + 1];
      r[kCpRecP + 2] = parent[3 * nd + 2];
    }
    static_assert(kCpRecP == 22 && kCpRecP + 3 <= kCpRecPad, "the record's parent at [22..24]");

    if (!std::getenv("NXHIP_CP_NOREC")) {
      CHECK(upload(&h->cp_rec, rec.data(), n * kCpRecPad, h->stream));
      if (!rng.empty()) CHECK(upload(&h->cp_rng, rng.data(), (int64_t)rng.size(), h->stream));
    }
    if (h->cp_rec == nullptr || h->cp_rng == nullptr) h->cp_runs.clear();
  }
  CHECK(dalloc(&h->cp_fac, std::max<int64_t>(1, E) * (h->N + 1) * (int64_t)kCpFac));
  // (several ranks: every rank's blocks by global edge, then the node rhs, summed)
  CHECK(dalloc(&h->cp_se, 20 * Es + (ranks ? 2 * n : 0)));
  if (ranks) {
    if (E > 0)
      CHECK(upload(&h->cp_gid, h->cp_gid_host.data(), E, h->stream));
    else
      CHECK(dalloc(&h->cp_gid, 1));
    CHECK(upload(&h->cp_nrowx, h->cp_nrowx_host.data(), 2 * n, h->stream));
  }
  CHECK(dalloc(&h->cp_xn, 2 * n));
  CHECK(dalloc(&h->cp_Pinv, 4 * n));
  CHECK(dalloc(&h->cp_hv, 2 * n));
  if (h->cp_rec) CHECK(dalloc(&h->cp_ctr, 6 * n));
  HIPCALL(hipStreamSynchronize(h->stream));
  h->cp_k = k;
  h->cp_m = m;
  h->cp_nI = nI;
  h->cp_nn = (int)n;
  h->cp_nlev = n_lev;
  h->cp_lev_host.assign(lev_off, lev_off + n_lev + 1);
  h->fe_cp = true;
  return NX_OK;
}

NX_API int nx_fe_set_direct(nx_network_t* h, nx_network_t* aux, int32_t k, int64_t n_lm,
                            const int32_t* slot, const int32_t* v_fe, const int32_t* v_aux,
                            const int32_t* i_fe, const int32_t* p_fe, const int32_t* p_aux,
                            const int32_t* l_fe, const int32_t* l_aux, const double* cst,
                            double ab) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (!h->fe) return fail(NX_ERR_STATE, "a general-degree handle (nx_create_fe)");
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  for (int** p : {&h->fe_slot, &h->fe_vfe, &h->fe_vaux, &h->fe_ife, &h->fe_pfe, &h->fe_paux,
                  &h->fe_lfe, &h->fe_laux}) {
    if (*p) HIPCALL(hipFree(*p));
    *p = nullptr;
  }
  if (h->fe_cst) HIPCALL(hipFree(h->fe_cst));
  h->fe_cst = nullptr;
  h->fe_aux = nullptr;
  if (aux == nullptr) return NX_OK;
  if (k < 2 || k > 16) return fail(NX_ERR_ARG, "flux degree k in 2..16");
  if (!slot || !v_fe || !v_aux || !i_fe || !p_fe || !p_aux || (n_lm > 0 && (!l_fe || !l_aux)) ||
      !cst)
    return fail(NX_ERR_ARG, "NULL array");
  if (aux->fe || !aux->pc || !aux->cond_mass || aux->N != h->N || aux->E != h->E ||
      (aux->n_cyc > 0 && !aux->cyc_team && (proc_rank(aux) || aux->nranks > 1)) ||
      aux->device != h->device ||
      aux->nranks != h->nranks ||
      aux->rank != h->rank || proc_rank(aux) != proc_rank(h) || aux->group || h->group)
    return fail(NX_ERR_STATE, "the auxiliary handle must be a P1/DG0 handle of the same "
                              "ranks with the same N and edges and its cell mass set "
                              "(nx_set_cell_mass); a graph with cycles (its Woodbury "
                              "correction, nx_set_cycles) on one rank");
  if (proc_rank(aux) &&
      !(aux->pc_lds && aux->pa.exact && aux->tree_exact && aux->pc_jobs > 0 &&
        aux->pa.n_coarse > 0 && aux->pa.n_coarse <= kCapCoarse))
    return fail(NX_ERR_STATE, "the auxiliary handle's ranks cannot run the direct tree solve "
                              "(LDS sweeps, exact forest, the coarse step)");
  const int64_t E = h->E, N = h->N, nv = E * (N + 1), np = E * N, km = k - 1;
  if (h->n_own != E * (k * N + 1 + N) + n_lm || aux->n_own != E * (2 * N + 1) + n_lm)
    return fail(NX_ERR_ARG, "row counts do not match a (k, 0) layout and its P1/DG0 one");
  auto in = [](const int32_t* a, int64_t n, int64_t lim) {
    for (int64_t i = 0; i < n; ++i)
      if (a[i] < 0 || a[i] >= lim) return false;
    return true;
  };
  if (!in(slot, E, E) || !in(v_fe, nv, h->n_own) || !in(i_fe, np * km, h->n_own) ||
      !in(p_fe, np, h->n_own) || !in(l_fe, n_lm, h->n_own) || !in(v_aux, nv, aux->n_own) ||
      !in(p_aux, np, aux->n_own) || !in(l_aux, n_lm, aux->n_own))
    return fail(NX_ERR_ARG, "row map out of range");
  int rc = NX_OK;
  if ((rc = upload(&h->fe_slot, slot, E, h->stream)) ||
      (rc = upload(&h->fe_vfe, v_fe, nv, h->stream)) ||
      (rc = upload(&h->fe_vaux, v_aux, nv, h->stream)) ||
      (rc = upload(&h->fe_ife, i_fe, np * km, h->stream)) ||
      (rc = upload(&h->fe_pfe, p_fe, np, h->stream)) ||
      (rc = upload(&h->fe_paux, p_aux, np, h->stream)) ||
      (rc = upload(&h->fe_lfe, l_fe, n_lm, h->stream)) ||
      (rc = upload(&h->fe_laux, l_aux, n_lm, h->stream)) ||
      (rc = upload(&h->fe_cst, cst, 4 * km + km * km, h->stream)))
    return rc;
  for (auto& e : h->fe_ev)
    if (!e) HIPCALL(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIPCALL(hipStreamSynchronize(h->stream));
  h->fe_aux = aux;
  h->fe_k = k;
  h->fe_nl = (int)n_lm;
  h->fe_ab = ab;
  return NX_OK;
}

NX_API int nx_set_pc_exact(nx_network_t* h, int32_t enable) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (!h->pc) return fail(NX_ERR_STATE, "nx_set_preconditioner(enable=1) must come first");
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  CHECK(drop_handle_graphs(h));
  h->pa.exact = enable ? 1 : 0;
  // direct_local() reads pa.exact: over RCCL the ranks' cached decision (direct_all, taken
  // in check_schedules) must be taken again
  h->sched_checked = false;
  return NX_OK;
}

NX_API int nx_set_solver(nx_network_t* h, int32_t solver, int32_t tree_exact) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (solver != 0 && solver != 1) return fail(NX_ERR_ARG, "solver: 0 = MINRES, 1 = direct");
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  h->solver = solver;
  h->tree_exact = tree_exact != 0;
  h->sched_checked = false;  // the solver choice is part of the ranks' schedule signature
  return NX_OK;
}

NX_API int nx_get_solver(nx_network_t* h, int32_t* requested, int32_t* last_run) {
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (requested) *requested = h->solver;
  if (last_run) *last_run = h->last_solver;
  return NX_OK;
}

NX_API int nx_set_lean(int32_t enable) {
  lean_flag() = enable ? 1 : 0;
  return NX_OK;
}

NX_API int nx_set_pc_kernels(nx_network_t* h, int32_t global) {
  if (!h) return fail(NX_ERR_ARG, "null handle");
  h->force_global = global ? 1 : 0;
  h->sched_checked = false;
  return NX_OK;
}

NX_API int nx_get_pc_kernels(nx_network_t* h, int32_t* lds) {
  if (!h || !lds) return fail(NX_ERR_ARG, "null argument");
  *lds = (h->pc && h->pc_lds) ? 1 : 0;
  return NX_OK;
}

NX_API int nx_get_pc_exact(nx_network_t* h, int32_t* enabled) {
  if (!h || !enabled) return fail(NX_ERR_ARG, "null argument");
  *enabled = h->pc ? h->pa.exact : 0;
  return NX_OK;
}

NX_API int nx_set_coarse(nx_network_t* h, int32_t n_coarse, const int32_t* slot_cidx,
                         int32_t n_cc, const int32_t* cc_chain, const int32_t* cc_top,
                         const int32_t* cc_bot, const int32_t* c_parent,
                         const int32_t* c_child_off, const int32_t* c_child, int32_t n_clvl,
                         const int32_t* c_lvl_off) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (!h->pc) return fail(NX_ERR_STATE, "nx_set_preconditioner(enable=1) must come first");
  if (n_coarse < 0 || n_cc < 0 || n_clvl < 0) return fail(NX_ERR_ARG, "negative sizes");
  if (n_coarse > kCapCoarse)
    return fail(NX_ERR_ARG, "coarse forest has " + std::to_string(n_coarse) + " junctions (cap " +
                                std::to_string(kCapCoarse) + ")");
  h->sched_checked = false;  // pa.lin / pa.fused change the exchange schedule
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  CHECK(drop_handle_graphs(h));
  const int64_t ns = h->pc_slots;
  if (n_coarse == 0) {
    h->pa.n_coarse = 0;
    return NX_OK;
  }
  if (!slot_cidx || !c_parent || !c_child_off || !c_lvl_off || (n_cc > 0 && (!cc_chain || !cc_top || !cc_bot)))
    return fail(NX_ERR_ARG, "null coarse array");
  // host copies of the top-level offsets to check that coarse slots sit in the top part
  std::vector<int> top_off(h->pa.n_top_lvl + 1);
  HIPCALL(hipMemcpy(top_off.data(), h->pa.top_lvl_off, sizeof(int) * top_off.size(),
                    hipMemcpyDeviceToHost));
  std::vector<int> lam(ns > 0 ? ns : 1);
  if (ns > 0) HIPCALL(hipMemcpy(lam.data(), h->pa.slot_lam, sizeof(int) * ns, hipMemcpyDeviceToHost));
  const int top0 = top_off[0], top1 = top_off.back();
  for (int64_t j = 0; j < ns; ++j) {
    if (slot_cidx[j] < -1 || slot_cidx[j] >= n_coarse) return fail(NX_ERR_ARG, "slot_cidx out of range");
    if (slot_cidx[j] >= 0 && (j < top0 || j >= top1))
      return fail(NX_ERR_ARG, "coarse slots must lie in the top part");
    if (lam[j] >= h->n_own && slot_cidx[j] < 0) return fail(NX_ERR_ARG, "ghost slot must be coarse");
  }
  for (int i = 0; i < n_cc; ++i)
    if (cc_chain[i] < 0 || cc_chain[i] >= h->E || cc_top[i] < 0 || cc_top[i] >= n_coarse ||
        cc_bot[i] < 0 || cc_bot[i] >= n_coarse)
      return fail(NX_ERR_ARG, "coarse chain out of range");
  if (c_child_off[0] != 0 || c_lvl_off[0] != 0 || c_lvl_off[n_clvl] != n_coarse)
    return fail(NX_ERR_ARG, "bad coarse offsets");
  for (int j = 0; j < n_coarse; ++j)
    if (c_parent[j] < -1 || c_parent[j] >= n_coarse) return fail(NX_ERR_ARG, "c_parent out of range");
  const int ncl = c_child_off[n_coarse];
  for (int i = 0; i < ncl; ++i)
    if (c_child[i] < 0 || c_child[i] >= n_coarse) return fail(NX_ERR_ARG, "c_child out of range");
  auto up = [&](const int32_t* src, int64_t n) -> const int* {
    int* d = nullptr;
    if (n <= 0) n = 1;
    if (hipMalloc((void**)&d, sizeof(int) * n) != hipSuccess) return nullptr;
    h->pc_bufs.push_back(d);
    if (src && hipMemcpy(d, src, sizeof(int) * n, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return d;
  };
  PcArgs& pa = h->pa;
  pa.slot_cidx = up(slot_cidx, ns);
  pa.cc_chain = up(n_cc ? cc_chain : nullptr, n_cc);
  pa.cc_top = up(n_cc ? cc_top : nullptr, n_cc);
  pa.cc_bot = up(n_cc ? cc_bot : nullptr, n_cc);
  pa.c_parent = up(c_parent, n_coarse);
  pa.c_child_off = up(c_child_off, n_coarse + 1);
  pa.c_child = up(ncl ? c_child : nullptr, ncl);
  pa.c_lvl_off = up(c_lvl_off, n_clvl + 1);
  {  // per coarse junction its chains in chain order (pc_coarse_partials)
    std::vector<int> off(n_coarse + 1, 0), ent;
    for (int i = 0; i < n_cc; ++i) {
      off[cc_top[i] + 1] += 1;
      off[cc_bot[i] + 1] += 1;
    }
    for (int k = 0; k < n_coarse; ++k) off[k + 1] += off[k];
    ent.assign(std::max(1, off[n_coarse]), 0);
    std::vector<int> fill(off.begin(), off.end() - 1);
    for (int i = 0; i < n_cc; ++i) {  // (a chain's top and bottom junctions differ)
      ent[fill[cc_top[i]]++] = i << 1;
      ent[fill[cc_bot[i]]++] = (i << 1) | 1;
    }
    pa.ck_off = up(off.data(), n_coarse + 1);
    pa.ck_ent = up(ent.data(), (int64_t)ent.size());
  }
  pa.c_wave = nullptr;
  if (n_coarse <= 64 && n_clvl <= 255) {  // coarse_wave_solve's packed set-up
    std::vector<int> cw(2 * std::max(1, (int)n_coarse), 0);
    bool ok = true;
    for (int lv = 0; lv < n_clvl && ok; ++lv)
      for (int j = c_lvl_off[lv]; j < c_lvl_off[lv + 1] && ok; ++j) {
        const int nk = c_child_off[j + 1] - c_child_off[j];
        if (nk > kWaveKids) {
          ok = false;
          break;
        }
        cw[2 * j] = lv | (nk << 8) | ((c_parent[j] + 1) << 12);
        int kids = 0;
        for (int k = 0; k < nk; ++k) kids |= c_child[c_child_off[j] + k] << (8 * k);
        cw[2 * j + 1] = kids;
      }
    if (ok) pa.c_wave = up(cw.data(), (int64_t)cw.size());
  }
  double* cb = nullptr;  // [D | J | G | alpha]
  HIPCALL(hipMalloc((void**)&cb, sizeof(double) * (3 * n_coarse + 1)));
  HIPCALL(hipMemset(cb, 0, sizeof(double) * (3 * n_coarse + 1)));
  h->pc_bufs.push_back(cb);
  pa.cbuf = cb;
  pa.xalpha = cb + 3 * n_coarse;
  pa.Gc = nullptr;
  if (n_coarse > 0 && n_coarse <= kCapCoarseLds) {
    {
      double* gc = nullptr;
      HIPCALL(hipMalloc((void**)&gc, sizeof(double) * n_coarse * n_coarse));
      HIPCALL(hipMemset(gc, 0, sizeof(double) * n_coarse * n_coarse));
      h->pc_bufs.push_back(gc);
      pa.Gc = gc;
    }
  }
  double* zc = nullptr;  // coarse solution (dense top with several ranks)
  HIPCALL(hipMalloc((void**)&zc, sizeof(double) * n_coarse));
  h->pc_bufs.push_back(zc);
  pa.zc = zc;
  // linear form needs the LDS kernels (the global-memory ones keep alpha's own all-reduce)
  pa.lin = h->pc_lds ? 1 : 0;
  // fused one-workgroup steps (k_pc_cpart in the up sweep's last workgroup, the coarse solve
  // in every down workgroup); the global-memory kernels keep the separate ones
  pa.fused = (h->pc_lds && h->pc_jobs > 0 && n_coarse <= kCapCoarseLds) ? 1 : 0;
  pa.fuse_pack = 0;  // set per solve path (solve_lean)
  {
    int* tk = nullptr;
    HIPCALL(hipMalloc((void**)&tk, 2 * sizeof(int)));
    HIPCALL(hipMemset(tk, 0, 2 * sizeof(int)));
    h->pc_bufs.push_back(tk);
    pa.ticket = tk;
  }
  for (const void* q : {(const void*)pa.slot_cidx, (const void*)pa.cc_chain, (const void*)pa.cc_top,
                        (const void*)pa.cc_bot, (const void*)pa.c_parent, (const void*)pa.c_child_off,
                        (const void*)pa.c_child, (const void*)pa.c_lvl_off})
    if (q == nullptr) return fail(NX_ERR_HIP, "coarse upload failed");
  pa.n_cc = n_cc;
  pa.n_clvl = n_clvl;
  pa.n_coarse = n_coarse;
  return NX_OK;
}

NX_API int nx_comm_unique_id(unsigned char* id_out) {
  if (!id_out) return fail(NX_ERR_ARG, "null argument");
  static_assert(sizeof(ncclUniqueId) == NX_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId id;
  NCCLCALL(ncclGetUniqueId(&id));
  std::memcpy(id_out, &id, sizeof(id));
  return NX_OK;
}

namespace {
// d_left_k: the cut index of every left row (the owned multiplier rows the down sweeps do
// not form), from the per-multiplier-row lm_cut of nx_set_cut
int build_left_cut(nx_network* h) {
  if (h->d_left_k) HIPCALL(hipFree(h->d_left_k));
  h->d_left_k = nullptr;
  std::vector<int> lk(std::max<size_t>(1, h->left_host.size()), -1);
  for (size_t i = 0; i < h->left_host.size(); ++i) {
    const int64_t m = h->left_host[i] - h->n_edge_dofs;
    if (m < 0 || m >= (int64_t)h->lm_cut.size()) return fail(NX_ERR_STATE, "left row outside the multiplier rows");
    lk[i] = h->lm_cut[m];
  }
  CHECK(upload(&h->d_left_k, lk.data(), (int64_t)lk.size(), h->stream));
  HIPCALL(hipStreamSynchronize(h->stream));
  return NX_OK;
}
}  // namespace

NX_API int nx_set_cut(nx_network_t* h, int32_t K, const int32_t* lm_cut, const int32_t* gk_off,
                      const int32_t* gk_row, const double* gk_coef) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null handle");
  if (K < 0 || (K > 0 && (!gk_off || (gk_off[K] > 0 && (!gk_row || !gk_coef)))))
    return fail(NX_ERR_ARG, "bad cut lists");
  const int64_t n_lm = h->n_own - h->n_edge_dofs;
  if (n_lm > 0 && !lm_cut) return fail(NX_ERR_ARG, "lm_cut needed for the multiplier rows");
  CHECK(set_device(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  CHECK(drop_handle_graphs(h));
  std::vector<int> own(std::max(1, (int)K), -1);
  for (int64_t m = 0; m < n_lm; ++m) {
    if (lm_cut[m] < -1 || lm_cut[m] >= K) return fail(NX_ERR_ARG, "lm_cut out of range");
    if (lm_cut[m] >= 0) {
      if (own[lm_cut[m]] >= 0) return fail(NX_ERR_ARG, "a cut index owned twice");
      own[lm_cut[m]] = (int)(h->n_edge_dofs + m);
    }
  }
  const int ne = K > 0 ? gk_off[K] : 0;
  for (int k = 0; k < K; ++k)
    if (gk_off[k] > gk_off[k + 1] || (own[k] >= 0 && gk_off[k + 1] > gk_off[k]))
      return fail(NX_ERR_ARG, "gk_off: an owned cut row takes no flux-end shares");
  for (int e = 0; e < ne; ++e)
    if (gk_row[e] < 0 || gk_row[e] >= h->n_edge_dofs) return fail(NX_ERR_ARG, "gk_row out of range");
  for (void* p : {(void*)h->d_cut_own, (void*)h->d_gk_off, (void*)h->d_gk_row,
                  (void*)h->d_gk_coef, (void*)h->cutbuf})
    if (p) HIPCALL(hipFree(p));
  h->d_cut_own = h->d_gk_off = h->d_gk_row = nullptr;
  h->d_gk_coef = h->cutbuf = nullptr;
  std::vector<int> off(gk_off ? gk_off : nullptr, gk_off ? gk_off + K + 1 : nullptr);
  if (off.empty()) off.assign(1, 0);
  std::vector<int> row(gk_row ? gk_row : nullptr, gk_row ? gk_row + ne : nullptr);
  std::vector<double> coef(gk_coef ? gk_coef : nullptr, gk_coef ? gk_coef + ne : nullptr);
  if (row.empty()) row.assign(1, 0);
  if (coef.empty()) coef.assign(1, 0.0);
  CHECK(upload(&h->d_cut_own, own.data(), (int64_t)own.size(), h->stream));
  CHECK(upload(&h->d_gk_off, off.data(), (int64_t)off.size(), h->stream));
  CHECK(upload(&h->d_gk_row, row.data(), (int64_t)row.size(), h->stream));
  CHECK(upload(&h->d_gk_coef, coef.data(), (int64_t)coef.size(), h->stream));
  CHECK(dalloc(&h->cutbuf, 2 + (int64_t)K));
  h->lm_cut.assign(lm_cut ? lm_cut : nullptr, lm_cut ? lm_cut + n_lm : nullptr);
  h->gk_off_host = off;
  h->gk_row_host.assign(gk_row ? gk_row : nullptr, gk_row ? gk_row + ne : nullptr);
  h->n_cut = K;
  h->sched_checked = false;  // the residual's exchange is part of the schedule signature
  if (!h->left_host.empty() || h->d_left) CHECK(build_left_cut(h));
  HIPCALL(hipStreamSynchronize(h->stream));
  return NX_OK;
}

NX_API int nx_set_halo(nx_network_t* h, int32_t nranks, int32_t rank, int32_t n_peers,
                       const int32_t* peer_rank, const int32_t* send_off,
                       const int32_t* send_idx, const int32_t* recv_off) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h) return fail(NX_ERR_ARG, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(NX_ERR_ARG, "bad rank/nranks");
  if (nranks > 1 && h->pc) return fail(NX_ERR_STATE, "set the halo plan before the preconditioner");
  if (nranks > 1 && h->fe && h->fe_cp && h->cp_Eg == 0)
    return fail(NX_ERR_STATE, "the halo plan before the continuous-pressure tables");
  if (n_peers < 0 || (n_peers > 0 && (!peer_rank || !send_off || !recv_off)))
    return fail(NX_ERR_ARG, "bad halo plan");
  CHECK(set_device(h));
  for (int i = 0; i < n_peers; ++i)
    if (peer_rank[i] < 0 || peer_rank[i] >= nranks || peer_rank[i] == rank)
      return fail(NX_ERR_ARG, "bad peer rank");
  h->peers.assign(peer_rank, peer_rank + n_peers);
  h->send_off.assign(send_off, send_off + n_peers + 1);
  h->recv_off.assign(recv_off, recv_off + n_peers + 1);
  if (n_peers == 0) {
    h->send_off.assign(1, 0);
    h->recv_off.assign(1, 0);
  }
  if (h->recv_off.back() != h->n_ghost)
    return fail(NX_ERR_ARG, "halo plan receives " + std::to_string(h->recv_off.back()) +
                                " values but the handle has " + std::to_string(h->n_ghost) +
                                " ghost columns");
  const int nsend = h->send_off.back();
  for (int i = 0; i < nsend; ++i)
    if (send_idx[i] < 0 || send_idx[i] >= h->n_own) return fail(NX_ERR_ARG, "send_idx out of range");
  if (h->send_idx) HIPCALL(hipFree(h->send_idx));
  if (h->send_buf) HIPCALL(hipFree(h->send_buf));
  h->send_idx = nullptr;
  h->send_buf = nullptr;
  CHECK(upload(&h->send_idx, send_idx, nsend, h->stream));
  CHECK(dalloc(&h->send_buf, nsend));
  if (h->gath) HIPCALL(hipFree(h->gath));
  h->gath = nullptr;
  CHECK(dalloc(&h->gath, nranks));
  HIPCALL(hipMemsetAsync(h->gath, 0, sizeof(double) * nranks, h->stream));
  h->beta_p2p = true;
  h->sched_checked = false;  // beta_p2p is part of the schedule signature
  h->nranks = nranks;
  h->rank = rank;
  h->have_plan = true;
  HIPCALL(hipStreamSynchronize(h->stream));
  return NX_OK;
}

NX_API int nx_comm_count(nx_network_t* h, int32_t* nranks) {
  if (!h || !nranks) return fail(NX_ERR_ARG, "null argument");
  if (!h->comm) {  // no RCCL communicator: the handle's own view (1, or a group's size)
    *nranks = h->nranks;
    return NX_OK;
  }
  int n = 0;
  NCCLCALL(ncclCommCount(h->comm, &n));
  *nranks = n;
  return NX_OK;
}

NX_API int nx_comm_init(nx_network_t* h, int32_t nranks, int32_t rank, const unsigned char* id,
                        int32_t n_peers, const int32_t* peer_rank, const int32_t* send_off,
                        const int32_t* send_idx, const int32_t* recv_off) {
  CHECK(flush_assembly(h));  // a deferred nx_assemble goes first
  if (!h || !id) return fail(NX_ERR_ARG, "null argument");
  if (h->group) return fail(NX_ERR_STATE, "the handle belongs to a group");
  CHECK(nx_set_halo(h, nranks, rank, n_peers, peer_rank, send_off, send_idx, recv_off));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  NCCLCALL(ncclCommInitRank(&h->comm, nranks, uid, rank));
  return NX_OK;
}

// Tests: nx_comm_init with the host transport in place of RCCL (several ranks' processes on
// one GPU, which RCCL refuses): `name` is a POSIX shared-memory name every rank passes (rank
// 0 chooses it, the host control plane broadcasts it). Eager collectives, no graphs.
NX_API int nx_comm_init_host(nx_network_t* h, int32_t nranks, int32_t rank, const char* name,
                             int32_t n_peers, const int32_t* peer_rank, const int32_t* send_off,
                             const int32_t* send_idx, const int32_t* recv_off) {
  CHECK(flush_assembly(h));
  if (!h || !name || name[0] != '/') return fail(NX_ERR_ARG, "a shared-memory name \"/...\"");
  if (h->group || proc_rank(h)) return fail(NX_ERR_STATE, "handle already has a transport");
  CHECK(nx_set_halo(h, nranks, rank, n_peers, peer_rank, send_off, send_idx, recv_off));
  CHECK(hc_open(name, nranks, rank, &h->hcomm));
  h->rccl_graph_ok = false;  // (every collective synchronises the stream: nothing is captured)
  return NX_OK;
}

namespace {
// The exchange step of ONE rank alone, its exchanges emulated (rehearsal of a multi-GPU run
// on one GPU, whose ranks cannot all be resident at once): the rank writes its slots into a
// scratch mailbox, and reads the sums the group's graph path left (cbuf; cutbuf) from slot 0
// of a mailbox whose other slots are zero and whose flags are set. Same work as the rank's
// launch in the real run, minus the wait for the others and the xGMI hops.
template <int W, int CPL>
int xr_rehearse_wc(nx_network* h, int P, double rtol, int reps, float* ms_out) {
  const size_t nb = xmb_bytes(P);
  void *rd = nullptr, *wr = nullptr;
  XPeer* dpeers = nullptr;
  int rc = NX_OK;
  auto cleanup = [&]() {
    if (rd) (void)hipFree(rd);
    if (wr) (void)hipFree(wr);
    if (dpeers) (void)hipFree(dpeers);
  };
  const unsigned tag = 0x7f000001u;
  {
    std::vector<double> img(nb / sizeof(double) + 1, 0.0);
    XPeer x = xpeer_of(img.data(), P);
    const int nC = h->pa.n_coarse, K = h->n_cut;
    if (hipMemcpy(x.mb1, h->pa.cbuf, sizeof(double) * 3 * nC, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(x.mb2, h->cutbuf, sizeof(double) * (2 + K), hipMemcpyDeviceToHost) != hipSuccess) {
      cleanup();
      return fail(NX_ERR_HIP, "rehearsal: reading the graph path's sums failed");
    }
    for (int k = 0; k < K; ++k) x.mb2[2 + k] = -x.mb2[2 + k];  // (the publisher forms 0 - sum)
    for (int i = 0; i < 2 * P; ++i) x.fl[i] = tag;
    const double tagd = __builtin_bit_cast(double, (unsigned long long)tag);
    for (int q = 0; q < P; ++q) {  // every slot carries its writer's tag
      x.mb1[(size_t)q * kXld1 + kXld1 - 1] = tagd;
      x.mb2[(size_t)q * kXld2 + kXld2 - 1] = tagd;
    }
    if (hipMalloc(&rd, nb) != hipSuccess || hipMalloc(&wr, nb) != hipSuccess ||
        hipMalloc((void**)&dpeers, sizeof(XPeer) * P) != hipSuccess ||
        hipMemcpy(rd, img.data(), nb, hipMemcpyHostToDevice) != hipSuccess) {
      cleanup();
      return fail(NX_ERR_HIP, "rehearsal: mailbox allocation failed");
    }
    std::vector<XPeer> peers(P, xpeer_of(wr, P));
    if (hipMemcpy(dpeers, peers.data(), sizeof(XPeer) * P, hipMemcpyHostToDevice) != hipSuccess) {
      cleanup();
      return fail(NX_ERR_HIP, "rehearsal: peer table upload failed");
    }
  }
  hipEvent_t e0, e1;
  HIPCALL(hipEventCreate(&e0));
  HIPCALL(hipEventCreate(&e1));
  for (const void* fn : {reinterpret_cast<const void*>(&k_dir_xr<W, CPL>),
                         reinterpret_cast<const void*>(&k_dir_xr<W, CPL, CPL <= 2>)})
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(160 * 1024 - xr_static_lds(h->dstep_variant)));
  (void)hipGetLastError();
  float total = 0.f;
  for (int k = 0; k <= reps && rc == NX_OK; ++k) {  // (launch 0: warm-up, not timed)
    DirStep da = dir_args(h, rtol);
    da.n_left = h->xr_nleft;
    da.xpeers = dpeers;
    da.xself = xpeer_of(rd, P);
    da.xP = P;
    da.xrank = h->rank;
    da.xld1 = kXld1;
    da.xld2 = kXld2;
    da.xK = h->n_cut;
    da.xtag = tag;
    if (sup_launch<CPL>(da))
      hipExtLaunchKernelGGL((k_dir_xr<W, CPL, CPL <= 2>), dim3(h->pc_jobs), dim3(kPcThreads),
                            h->dstep_lds, h->stream, e0, e1, 0, h->pa, da);
    else
      hipExtLaunchKernelGGL((k_dir_xr<W, CPL>), dim3(h->pc_jobs), dim3(kPcThreads), h->dstep_lds,
                            h->stream, e0, e1, 0, h->pa, da);
    if (hipGetLastError() != hipSuccess) rc = fail(NX_ERR_HIP, "rehearsal launch failed");
    h->dstep_epoch += 1;
    h->seq += 1;
    if (rc == NX_OK) rc = wait_published(h);
    float ms = 0.f;
    if (rc == NX_OK && hipEventSynchronize(e1) == hipSuccess &&
        hipEventElapsedTime(&ms, e0, e1) == hipSuccess && k > 0)
      total += ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamSynchronize(h->stream);
  cleanup();
  if (rc == NX_OK) *ms_out = total / (float)std::max(reps, 1);
  return rc;
}
}  // namespace

// Test / rehearsal hook (no reference counterpart): the exchange step of rank h of a group
// alone, reps timed launches (HIP events bound to the dispatch), its exchanges emulated from
// the sums of the group's previous graph-path direct solve (scripts/group_rehearsal.py).
// The solution left in h's x is the rank's share of the real answer.
NX_API int nx_debug_xr_rehearse(nx_network_t* h, double rtol, int32_t reps, double* ms) {
  if (!h || !ms) return fail(NX_ERR_ARG, "null argument");
  if (!h->group) return fail(NX_ERR_STATE, "a group member (its graph path solved first)");
  if (!h->xr_ok || !xr_variant(h->dstep_variant) || h->pa.n_coarse <= 0 || h->n_cut < 0 ||
      h->pa.n_coarse > kCapCoarseLds || h->n_cut > kCapCoarseLds)
    return fail(NX_ERR_STATE, "this rank cannot run the exchange step");
  CHECK(set_device(h));
  float v = 0.f;
  int rc;
  switch (h->dstep_variant) {
    case 5: rc = xr_rehearse_wc<8, 2>(h, h->nranks, rtol, reps, &v); break;
    case 7: rc = xr_rehearse_wc<8, 4>(h, h->nranks, rtol, reps, &v); break;
    case 10: rc = xr_rehearse_wc<8, 3>(h, h->nranks, rtol, reps, &v); break;
    default: rc = xr_rehearse_wc<16, 4>(h, h->nranks, rtol, reps, &v); break;
  }
  *ms = v;
  return rc;
}

// The RCCL ranks' shape of the exchange step on one GPU: every rank of the group launches its
// own k_dir_xr (a one-handle team, no group: the exchange width is the handle's nranks) on a
// stream of its own, so the launches run concurrently and meet only through the mailboxes,
// as on separate GPUs. The ranks' assembly must be pending (nx_assemble); their jobs must fit
// the GPU together (co-resident). The outcome is settled as the group's one launch settles it
// (xr_conclude); a step the ranks did not finish is solved again on the group's graph path. *relres: the published residual (every rank's equal).
NX_API int nx_debug_xr_separate(nx_group_t* g, double rtol, double* relres) {
  if (!g || !relres) return fail(NX_ERR_ARG, "null argument");
  const int P = g->P;
  int jobs = 0;
  for (nx_network* h : g->hs) {
    if (!xr_local(h) || !h->pend_lhs || !h->pend_rhs || h->xr_off)
      return fail(NX_ERR_STATE, "every rank able to run the exchange step, its assembly pending");
    jobs += h->pc_jobs;
  }
  if (jobs > g->hs[0]->n_cu) return fail(NX_ERR_STATE, "the ranks' jobs do not fit the GPU together");
  CHECK(set_device(g->hs[0]));
  HIPCALL(hipStreamSynchronize(g->stream));
  std::vector<hipStream_t> ss(P, nullptr);
  for (int r = 0; r < P; ++r) HIPCALL(hipStreamCreateWithFlags(&ss[r], hipStreamNonBlocking));
  for (int r = 0; r < P; ++r) g->hs[r]->stream = ss[r];
  int rc = NX_OK;
  for (int r = 0; r < P && rc == NX_OK; ++r) rc = launch_xr(Team{&g->hs[r], 1, nullptr}, rtol);
  int outcome = kXrGraph;
  if (rc == NX_OK) rc = xr_conclude(g->hs.data(), P, true, rtol, &outcome);
  for (int r = 0; r < P; ++r) (void)hipStreamSynchronize(ss[r]);
  for (int r = 0; r < P; ++r) {
    g->hs[r]->stream = g->stream;
    (void)hipStreamDestroy(ss[r]);
  }
  CHECK(rc);
  if (outcome == kXrDone) {
    for (nx_network* h : g->hs) h->last_solver = 1;
    *relres = g->hs[0]->h_last->relres;
    return NX_OK;
  }
  int32_t it = 0, conv = 0;  // (given up everywhere, or above rtol: the group's graph path)
  CHECK(solve_team(Team{g->hs.data(), P, g}, rtol, 1 << 16, 4, &it, relres, &conv));
  return NX_OK;
}

// Test hook: the poll bound of this rank's exchange `which` (0: the coarse partials, 1: the
// residual) in its next exchange steps; 0 makes that exchange give up at once (after this
// rank's own slots and flags are written, so the others may still finish it).
NX_API int nx_debug_xr_polls(nx_network_t* h, int32_t which, uint32_t polls) {
  if (!h || which < 0 || which > 1) return fail(NX_ERR_ARG, "which is 0 or 1");
  h->xpoll[which] = polls;
  return NX_OK;
}

// [xr_off, the last launch's give-up reasons (kXrFail*), agreements taken part in, the last
// launch's tag]
NX_API int nx_get_xr_status(nx_network_t* h, int32_t* out) {
  if (!h || !out) return fail(NX_ERR_ARG, "null argument");
  out[0] = h->xr_off ? 1 : 0;
  out[1] = (int32_t)h->xr_why;
  out[2] = h->xr_agreed;
  out[3] = (int32_t)h->xtag;
  return NX_OK;
}

NX_API int nx_xch_export(nx_network_t* h, unsigned char* handle_out) {
  if (!h || !handle_out) return fail(NX_ERR_ARG, "null argument");
  if (!proc_rank(h)) return fail(NX_ERR_STATE, "nx_comm_init first");
  CHECK(set_device(h));
  CHECK(xr_alloc(h, h->nranks));
  hipIpcMemHandle_t m;
  HIPCALL(hipIpcGetMemHandle(&m, h->xmb));
  static_assert(sizeof(hipIpcMemHandle_t) <= NX_XCH_HANDLE_BYTES, "IPC handle size");
  std::memset(handle_out, 0, NX_XCH_HANDLE_BYTES);
  std::memcpy(handle_out, &m, sizeof(m));
  return NX_OK;
}

NX_API int nx_xch_import(nx_network_t* h, const unsigned char* handles) {
  if (!h || !handles) return fail(NX_ERR_ARG, "null argument");
  if (!proc_rank(h) || !h->xmb) return fail(NX_ERR_STATE, "nx_xch_export first");
  CHECK(set_device(h));
  const int P = h->nranks;
  std::vector<XPeer> peers(P);
  for (int q = 0; q < P; ++q) {
    if (q == h->rank) {
      peers[q] = xpeer_of(h->xmb, P);
      continue;
    }
    hipIpcMemHandle_t m;
    std::memcpy(&m, handles + (size_t)q * NX_XCH_HANDLE_BYTES, sizeof(m));
    void* ptr = nullptr;
    HIPCALL(hipIpcOpenMemHandle(&ptr, m, hipIpcMemLazyEnablePeerAccess));
    h->xr_opened.push_back(ptr);
    peers[q] = xpeer_of(ptr, P);
  }
  return xr_link(h, peers);
}

NX_API int nx_group_create(int32_t nranks, nx_network_t* const* handles, nx_group_t** out) {
  if (!out || !handles) return fail(NX_ERR_ARG, "null argument");
  *out = nullptr;
  if (nranks < 1 || nranks > kMaxGroup)
    return fail(NX_ERR_ARG, "group size must be 1.." + std::to_string(kMaxGroup));
  for (int r = 0; r < nranks; ++r) {
    nx_network* h = handles[r];
    if (!h) return fail(NX_ERR_ARG, "null handle in group");
    // (a deferred nx_assemble stays pending: the group's first direct solve runs it inside
    // its own launch, on the group's stream)
    if (h->group || proc_rank(h)) return fail(NX_ERR_STATE, "handle already has a transport");
    if (h->device != handles[0]->device) return fail(NX_ERR_ARG, "group members share one device");
    if (nranks > 1 && (!h->have_plan || h->rank != r || h->nranks != nranks))
      return fail(NX_ERR_STATE, "handle " + std::to_string(r) + " needs nx_set_halo(rank " +
                                    std::to_string(r) + " of " + std::to_string(nranks) + ")");
  }
  // where each ghost segment comes from: my segment in the peer's send buffer
  for (int r = 0; r < nranks; ++r) {
    nx_network* h = handles[r];
    h->peer_src_off.assign(h->peers.size(), 0);
    for (size_t j = 0; j < h->peers.size(); ++j) {
      nx_network* p = handles[h->peers[j]];
      const auto it = std::find(p->peers.begin(), p->peers.end(), r);
      const int cnt = h->recv_off[j + 1] - h->recv_off[j];
      if (it == p->peers.end()) {
        if (cnt > 0) return fail(NX_ERR_ARG, "halo plans disagree (missing peer)");
        continue;
      }
      const size_t i = (size_t)(it - p->peers.begin());
      if (p->send_off[i + 1] - p->send_off[i] != cnt)
        return fail(NX_ERR_ARG, "halo plans disagree: rank " + std::to_string(h->peers[j]) +
                                    " sends " + std::to_string(p->send_off[i + 1] - p->send_off[i]) +
                                    " values, rank " + std::to_string(r) + " expects " +
                                    std::to_string(cnt));
      h->peer_src_off[j] = p->send_off[i];
    }
  }
  HIPCALL(hipSetDevice(handles[0]->device));
  auto* g = new nx_group();
  g->P = nranks;
  g->hs.assign(handles, handles + nranks);
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
    delete g;
    return fail(NX_ERR_HIP, "hipStreamCreate failed");
  }
  for (nx_network* h : g->hs) {
    (void)hipStreamSynchronize(h->stream);
    h->own_stream = h->stream;
    h->stream = g->stream;
    h->group = g;
  }
  // the exchange step's mailboxes (k_dir_xg): each rank writes into every rank's own
  if (nranks > 1) {
    std::vector<XPeer> peers(nranks);
    int rc = NX_OK;
    for (int r = 0; r < nranks && rc == NX_OK; ++r) rc = xr_alloc(g->hs[r], nranks);
    for (int r = 0; r < nranks && rc == NX_OK; ++r) peers[r] = xpeer_of(g->hs[r]->xmb, nranks);
    for (int r = 0; r < nranks && rc == NX_OK; ++r) rc = xr_link(g->hs[r], peers);
    if (rc != NX_OK)  // (no exchange step: the graph path)
      for (nx_network* h : g->hs) xr_free(h);
  }
  *out = g;
  return NX_OK;
}

NX_API int nx_group_solve(nx_group_t* g, double rtol, int32_t maxit, int32_t check_every,
                          int32_t* iters, double* relres, int32_t* converged) {
  if (!g) return fail(NX_ERR_ARG, "null group");
  return solve_team(Team{g->hs.data(), g->P, g}, rtol, maxit, check_every, iters, relres, converged);
}

NX_API int nx_group_destroy(nx_group_t* g) {
  if (!g) return NX_OK;
  (void)hipSetDevice(g->hs[0]->device);
  (void)hipStreamSynchronize(g->stream);
  (void)drop_graph(GraphSlot{&g->chunk_exec, &g->chunk_graph, &g->chunk_len, &g->lean});
  for (nx_network* h : g->hs) {
    h->stream = h->own_stream;
    h->own_stream = nullptr;
    h->group = nullptr;
    xr_free(h);  // (the peers were the group's)
  }
  if (g->xg_dev) (void)hipFree(g->xg_dev);
  if (g->xg_host) (void)hipHostFree(g->xg_host);
  (void)hipStreamDestroy(g->stream);
  delete g;
  return NX_OK;
}

#ifdef NX_PHASE_TIMING
NX_API int nx_debug_phases(unsigned long long* out, int32_t n) {
  if (!out || n < 1 || n > 128) return fail(NX_ERR_ARG, "bad argument");
  HIPCALL(hipDeviceSynchronize());
  HIPCALL(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * n));
  return NX_OK;
}

NX_API int nx_debug_dstep(unsigned long long* out) {  // 48 x 512 stamps of k_dir_step
  HIPCALL(hipDeviceSynchronize());
  HIPCALL(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dst), sizeof(unsigned long long) * 48 * 512));
  return NX_OK;
}

NX_API int nx_debug_wg(unsigned long long* starts, unsigned long long* ends) {
  HIPCALL(hipDeviceSynchronize());
  HIPCALL(hipMemcpyFromSymbol(starts, HIP_SYMBOL(g_wgs), sizeof(unsigned long long) * 8 * 512));
  HIPCALL(hipMemcpyFromSymbol(ends, HIP_SYMBOL(g_wge), sizeof(unsigned long long) * 8 * 512));
  return NX_OK;
}
#endif
