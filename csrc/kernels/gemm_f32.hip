// fp32 GEMM on the CDNA4 f32-input matrix cores (v_mfma_f32_32x32x2_f32), for the convolutions of
// the fp32 training step (the reference harness's precision: examples/torch/
// pytorch_synthetic_benchmark.py:86 trains torchvision ResNet-50 in fp32).
//
//   C[m][n] (+)= sum_k A(m, k) * B(n, k)          exact f32 (an fmaf chain per output, no xf32)
//
// Each operand is either K-CONTIGUOUS (X(r, k) = x[r*ld + k]) or MN-CONTIGUOUS (X(r, k) =
// x[k*ld + r]), which covers the three GEMMs of a 1x1 convolution over channels_last
// activations [M = N*H*W, C]:
//   forward        Y[M][Cout]  = X[M][Cin] . W[Cout][Cin]^T       A K-contig, B K-contig
//   backward-data  dX[M][Cin]  = dY[M][Cout] . W[Cout][Cin]       A K-contig, B MN-contig
//   weight grad    dW[Cout][Cin] = dY^T . X  (K = M, split-K)     A MN-contig, B MN-contig
//
// Tiling for 64-wide waves: a 256-thread workgroup owns a BM x BN tile (128x128, 128x64 or
// 64x128) as a 2x2 grid of waves, each wave a (BM/2)x(BN/2) grid of 32x32 MFMA blocks with f32x16
// accumulators.  K advances in BK = 32 slices through two LDS stages (one barrier per slice:
// the next slice's global loads are in flight while the MFMAs consume the current one).
//   LDS images:  K-contig operand  [r][k], rows of 36 floats: 16-B stores of the 16-B global
//                loads, and ONE ds_read_b128 per lane per 8-k group (conflict-free: the 4-float
//                pad spreads the 16 lanes of each b128 group over all 64 banks)
//                MN-contig operand [k][r]: 16-B stores, four ds_read_b32 per 8-k group
//                (32 consecutive r per half-wave: conflict-free)
// The k order inside an 8-k group is permuted per lane half -- the MFMA slot k=h of step s takes
// actual k = 8g + 4h + s -- identically for A and B, so each lane's 4 operands of a group are 4
// consecutive k (the single 16-B read) and the sum is unchanged.
// Blocks are remapped so each XCD (blocks are dealt round-robin to the 8 XCDs) walks a contiguous
// run of tiles, n fastest: neighbouring tiles share A rows in that XCD's L2.
// Split-K (weight gradients: K = N*H*W up to 10^5 against a small output) accumulates with f32
// atomics into a zeroed C.
//
// 3x3 convolutions (pad 1) run on the SAME kernel as implicit GEMMs: no im2col buffer, the
// operand loader gathers the shifted NHWC pixels straight from the activation (zero outside the
// image), with the weight in its channels_last image [Cout][3][3][Cin] (k = tap * C + c):
//   forward      Y[(n,oy,ox)][co]  = sum_(tap,ci) x[n, s*oy+dy, s*ox+dx, ci] . W[co][tap][ci]
//                A = implicit rows (mode 2), B = W K-contig (ld = 9 Cin)
//   data grad    dX[(n,iy,ix)][ci] = sum_(tap,co) dY[n, iy-dy, ix-dx, co] . W[co][tap][ci]   (stride 1)
//                A = implicit rows, flipped taps (mode 2), B = W per tap MN-contig (mode 4)
//   weight grad  dW[co][(tap,ci)]  = sum_(n,oy,ox) dY[(n,oy,ox)][co] . x[n, s*oy+dy, s*ox+dx, ci]
//                A = dY MN-contig, B = implicit MN rows (tap, ci) over k = output pixels (mode 3)
// A BK = 32 k-slice never straddles a tap (C % 32 == 0 for the K-contig gathers), so the shift is
// uniform per slice and each row costs one bounds test per slice.
#include <algorithm>

#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kGB = 256;  // threads per workgroup (4 waves)
// k per LDS stage: 32 (4 x 8-k groups; BK = 16 with 4 workgroups per CU measured slower).  The
// round-4 64-k-slice variant (tile codes 5-7, 70-104 KB of static LDS) is gone: it won no
// direction in situ by more than 1 us (profiles/r4_autotune_decisions.txt) and coincided with
// aborts in forked captures that were never root-caused; the small-M layers get their extra
// workgroups from split-K instead (ops/conv.py C3_SPLIT_BACKENDS).
constexpr int BK = 32;

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct GemmParams {
  const float* A;
  const float* B;
  float* C;
  int M, N, K;
  int64_t lda, ldb, ldc;
  int tiles_m, tiles_n, splits, k_per_split;
  int atomic;
  int c_vec;  // C rows 16-B aligned (ldc % 4 == 0, C 16-B aligned): float4 stores
  float* stats;  // optional (non-split GEMMs): per (row tile, column) [sum | sum of squares] of C,
                 // [tiles_m][2][N] -- the BatchNorm statistics of a conv output, fused
  // implicit-GEMM convolution geometry (modes 2-4)
  int gHr, gWr;        // pixel grid of the implicit rows (mode 2) / of k (mode 3)
  int gHs, gWs;        // grid of the gathered activation
  int gC;              // its channels (k per tap, mode 2; rows per tap, mode 3)
  int gS, gSign;       // row / k pixel -> source pixel: s * (y, x) + sign * (dy, dx)
  int gT;              // taps per side: 3 (3x3, pad 1) or 1 (1x1, pad 0)
  float gInvWr, gInvHr;
  int kt;              // mode 4: k per tap (Cout)
  int64_t tap_off;     // mode 4: element offset between the taps of a weight row (Cin)
  // BatchNorm-backward epilogue (with stats): C is the gradient dy of a BN(+ReLU) output whose
  // input x, ReLU mask bits and forward save (mean [N], invstd [N] at +N) are given; the epilogue
  // writes per (row tile, column) [sum dz | sum dz * (x - mean)], dz = dy masked by the ReLU --
  // the BN backward's reduction pass over (dy, x) disappears (ops/bnact.py hand-off)
  const float* bx;
  const uint8_t* bmask;  // null: no ReLU mask (brelu: recomputed from x and the save's scale / shift)
  const float* bsave;
  int brelu;
  // BatchNorm-apply prologue: the operand `xop` (1 = A, 2 = B) is a BN INPUT x whose output
  // act(scale[c] * x + shift[c]) (scale / shift at xsave + 2C / + 3C) is what the GEMM multiplies
  // -- transformed as it is loaded (the image's zero padding stays zero); the BN output is never
  // written to memory (ops/conv.py _BnActConvFn)
  const float* xsave;
  int xC, xrelu, xop;
};

__host__ __device__ constexpr int bnb_slots(int nr) { return nr > 0 ? nr : 1; }

__device__ __forceinline__ float4 bn_xform(float4 v, float4 sc, float4 sh, int relu) {
  v = make_float4(fmaf(v.x, sc.x, sh.x), fmaf(v.y, sc.y, sh.y), fmaf(v.z, sc.z, sh.z), fmaf(v.w, sc.w, sh.w));
  if (relu) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
  return v;
}

// Operand modes.  0: K-contig rows, 1: MN-contig, 2: implicit conv rows (K-contig gather of
// shifted pixels), 3: implicit conv MN rows (r = tap * C + c, k = output pixel), 4: a 3x3 weight
// per tap, MN-contig (r = ci, k = tap * kt + co)
__host__ __device__ constexpr bool mode_kc(int mode) { return mode == 0 || mode == 2; }

// m = q * d + r with 0 <= r < d for m < 2^24 (one float multiply and one correction step)
__device__ __forceinline__ int fdivmod(int m, int d, float inv, int* r) {
  int q = (int)((float)m * inv);
  int rr = m - q * d;
  if (rr < 0) {
    --q;
    rr += d;
  } else if (rr >= d) {
    ++q;
    rr -= d;
  }
  *r = rr;
  return q;
}

template <int R, int MODE>
struct Operand {
  static constexpr int LDK = BK + 4;                   // K-contig row pitch (conflict-free b128 reads)
  static constexpr bool KC = mode_kc(MODE);
  static constexpr int NV = R * BK / 4 / kGB;          // float4 per thread per stage
  static constexpr int LDS = KC ? R * LDK : BK * R;    // floats per stage
  static constexpr int TPR = R / 4;                    // MN-contig: threads per k row
  float4 v[NV];
  // mode 2: per row of this thread, the source pixel of tap (0, 0) and the image base row
  int sy[MODE == 2 ? NV : 1], sx[MODE == 2 ? NV : 1], pn[MODE == 2 ? NV : 1];
  // mode 3: this thread's (fixed) row r = tap * C + c
  int rdy, rdx, rc;
  bool rok;
  // modes 2 / 4: (tap, offset inside the tap) of the NEXT k-slice to load, advanced by BK per load
  // (slices are loaded strictly in order) -- no per-stage integer division: a division by a
  // runtime value is ~40 scalar instructions, and two per stage made the 3x3 implicit GEMMs issue
  // 4x the scalar instructions of MIOpen's solvers (profiles/r5_c3_pmc.txt)
  int ltap, lc, lty, ltx;
  // mode 3: output pixel (n, oy, ox) of each of this thread's k rows of the NEXT slice, advanced by
  // BK = (dn, doy, dox) pixels per load with one conditional carry each (no per-element division)
  int kn[MODE == 3 ? NV : 1], koy[MODE == 3 ? NV : 1], kox[MODE == 3 ? NV : 1];
  int dn, doy, dox;
  bool xf;           // BN-apply prologue on this operand
  float4 xsc, xsh;   // the channels' scale / shift: fixed rows (MN modes) or this slice's k (KC)
  uint32_t xok;      // bit i: v[i] was loaded (transformed at store; padding / out of range stays 0)
  int xrelu;

  __device__ __forceinline__ void init(const GemmParams& p, int r0, int rmax, int which, int kb) {
    xf = p.xsave != nullptr && p.xop == which;
    xrelu = p.xrelu;
    xok = 0;
    if constexpr (MODE == 2 || MODE == 4) {  // one division per workgroup (the split's first slice)
      const int per = MODE == 2 ? p.gC : p.kt;
      ltap = kb / per;
      lc = kb - ltap * per;
      lty = ltap / 3;
      ltx = ltap - 3 * lty;
    }
    if (xf && !KC) {  // rows are channels (mode 1: r; mode 3: rc), fixed per thread
      int c = r0 + 4 * (threadIdx.x % TPR);
      if constexpr (MODE == 3) c = (c < rmax ? c : 0) % p.gC;
      if (c + 3 >= p.xC) c = 0;
      xsc = *reinterpret_cast<const float4*>(p.xsave + 2 * p.xC + c);
      xsh = *reinterpret_cast<const float4*>(p.xsave + 3 * p.xC + c);
    }
    if constexpr (MODE == 2) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int r = r0 + threadIdx.x / (BK / 4) + (kGB / (BK / 4)) * i;
        int x, y;
        const int q = fdivmod(r < rmax ? r : 0, p.gWr, p.gInvWr, &x);
        const int n = fdivmod(q, p.gHr, p.gInvHr, &y);
        sy[i] = r < rmax ? y * p.gS : -(1 << 20);  // invalid rows fail every bounds test
        sx[i] = x * p.gS;
        pn[i] = n * p.gHs;
      }
    } else if constexpr (MODE == 3) {
      const int hw = p.gHr * p.gWr;
      dn = BK / hw;
      doy = (BK - dn * hw) / p.gWr;
      dox = BK - dn * hw - doy * p.gWr;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int k = kb + threadIdx.x / TPR + (kGB / TPR) * i;
        int ox, oy;
        const int q = fdivmod(k, p.gWr, p.gInvWr, &ox);
        kn[i] = fdivmod(q, p.gHr, p.gInvHr, &oy);
        koy[i] = oy;
        kox[i] = ox;
      }
      const int r = r0 + 4 * (threadIdx.x % TPR);
      rok = r < rmax;
      const int tap = r / p.gC;
      rc = r - tap * p.gC;
      rdy = p.gT == 3 ? tap / 3 - 1 : 0;  // 3x3 pad 1, or 1x1 pad 0 (strided)
      rdx = p.gT == 3 ? tap % 3 - 1 : 0;
    }
  }

  __device__ __forceinline__ void load(const GemmParams& p, const float* __restrict__ x, int64_t ld, int r0, int rmax,
                                       int k0, int kmax) {
    if constexpr (MODE == 2) {
      // tap (uniform over the slice: C % BK == 0) from the running state, then advance it
      const int dy = p.gT == 3 ? (lty - 1) * p.gSign : 0, dx = p.gT == 3 ? (ltx - 1) * p.gSign : 0;
      const int c = lc + 4 * (threadIdx.x % (BK / 4));
      advance(p.gC);
      if (xf) {  // consumed at store(): the loads stay in flight across the MFMAs
        xsc = *reinterpret_cast<const float4*>(p.xsave + 2 * p.xC + c);
        xsh = *reinterpret_cast<const float4*>(p.xsave + 3 * p.xC + c);
        xok = 0;
      }
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int iy = sy[i] + dy, ix = sx[i] + dx;
        v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((unsigned)iy < (unsigned)p.gHs && (unsigned)ix < (unsigned)p.gWs && k0 < kmax) {
          // 32-bit element index (the binding checks every operand has < 2^31 elements)
          v[i] = *reinterpret_cast<const float4*>(x + (uint32_t)(((pn[i] + iy) * p.gWs + ix) * p.gC + c));
          xok |= 1u << i;  // outside the image: the padding's 0, never transformed
        }
      }
      return;
    }
    if constexpr (MODE == 0) {  // channels = k (per slice)
      if (xf) {
        const int c = k0 + 4 * (threadIdx.x % (BK / 4));
        xsc = xsh = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c + 3 < p.xC) {
          xsc = *reinterpret_cast<const float4*>(p.xsave + 2 * p.xC + c);
          xsh = *reinterpret_cast<const float4*>(p.xsave + 3 * p.xC + c);
        }
      }
    }
    xok = 0;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int r, k;
      if constexpr (KC) {
        r = r0 + threadIdx.x / (BK / 4) + (kGB / (BK / 4)) * i;
        k = k0 + 4 * (threadIdx.x % (BK / 4));
      } else {
        r = r0 + 4 * (threadIdx.x % TPR);
        k = k0 + threadIdx.x / TPR + (kGB / TPR) * i;
      }
      v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (MODE == 3) {
        const int n = kn[i], oy = koy[i], ox = kox[i];
        {  // advance this k row to the next slice: + BK pixels
          int nx = ox + dox, ny = oy + doy, nn = n + dn;
          if (nx >= p.gWr) {
            nx -= p.gWr;
            ++ny;
          }
          if (ny >= p.gHr) {
            ny -= p.gHr;
            ++nn;
          }
          kn[i] = nn;
          koy[i] = ny;
          kox[i] = nx;
        }
        if (rok && k < kmax) {
          const int iy = oy * p.gS + rdy, ix = ox * p.gS + rdx;
          if ((unsigned)iy < (unsigned)p.gHs && (unsigned)ix < (unsigned)p.gWs) {
            v[i] = *reinterpret_cast<const float4*>(x + (uint32_t)(((n * p.gHs + iy) * p.gWs + ix) * p.gC + rc));
            xok |= 1u << i;
          }
        }
      } else if constexpr (MODE == 4) {
        if (r < rmax && k < kmax)  // tap uniform over the slice (kt % BK == 0): the running state
          v[i] = *reinterpret_cast<const float4*>(x + (uint32_t)(ltap * (int)p.tap_off + (lc + (k - k0)) * (int)ld + r));
      } else if (r < rmax && k < kmax) {
        v[i] = KC ? *reinterpret_cast<const float4*>(x + (int64_t)r * ld + k)
                  : *reinterpret_cast<const float4*>(x + (int64_t)k * ld + r);
        xok |= 1u << i;
      }
    }
    if constexpr (MODE == 4) advance(p.kt);
  }
  __device__ __forceinline__ void advance(int per) {
    lc += BK;
    if (lc >= per) {
      lc -= per;
      ++ltap;
      if (++ltx == 3) {
        ltx = 0;
        ++lty;
      }
    }
  }
  __device__ __forceinline__ void store(float* lds) {
    if (xf) {  // BN-apply prologue, applied here so the stage's global loads overlap the MFMAs
#pragma unroll
      for (int i = 0; i < NV; ++i)
        if ((xok >> i) & 1u) v[i] = bn_xform(v[i], xsc, xsh, xrelu);
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if constexpr (KC) {
        const int r = threadIdx.x / (BK / 4) + (kGB / (BK / 4)) * i, k = 4 * (threadIdx.x % (BK / 4));
        *reinterpret_cast<float4*>(lds + r * LDK + k) = v[i];
      } else {
        const int r = 4 * (threadIdx.x % TPR), k = threadIdx.x / TPR + (kGB / TPR) * i;
        *reinterpret_cast<float4*>(lds + k * R + r) = v[i];
      }
    }
  }
  // the lane's 4 operands of 8-k group g: k = 8g + 4h + s, s = 0..3, row r
  __device__ __forceinline__ float4 frag(const float* lds, int r, int g, int h) const {
    const int k = 8 * g + 4 * h;
    if constexpr (KC) {
      return *reinterpret_cast<const float4*>(lds + r * LDK + k);
    } else {
      return make_float4(lds[k * R + r], lds[(k + 1) * R + r], lds[(k + 2) * R + r], lds[(k + 3) * R + r]);
    }
  }
};

__device__ __forceinline__ float f4get(const float4& v, int s) { return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w; }

template <int BM, int BN, int AM, int BMD>
__global__ __launch_bounds__(kGB, 2) void gemm_f32_kernel(GemmParams p) {
  using OA = Operand<BM, AM>;
  using OB = Operand<BN, BMD>;
  constexpr int STAGE = OA::LDS + OB::LDS;
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 32, FN = WN / 32;
  constexpr int CP = WN + 4;                  // padded row pitch of a wave's staged 32-row C slab
  constexpr int CSTAGE = 4 * 32 * CP;        // the 4 waves' slabs (epilogue)
  constexpr int LDS_TOTAL = 2 * STAGE > CSTAGE ? 2 * STAGE : CSTAGE;
  __shared__ __align__(16) float lds[LDS_TOTAL];

  int b = blockIdx.x;
  const int nb = gridDim.x;
  if ((nb & 7) == 0) b = (b & 7) * (nb >> 3) + (b >> 3);  // XCD-contiguous tile runs
  const int split = b % p.splits;
  const int t = b / p.splits;
  const int tn = t % p.tiles_n, tm = t / p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kb = split * p.k_per_split;
  const int ke = min(p.K, kb + p.k_per_split);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w & 1, wn = w >> 1;
  const int lr = lane & 31, lh = lane >> 5;

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  OA oa;
  OB ob;
  oa.init(p, m0, p.M, 1, kb);
  ob.init(p, n0, p.N, 2, kb);
  if (kb < ke) {
    oa.load(p, p.A, p.lda, m0, p.M, kb, ke);
    ob.load(p, p.B, p.ldb, n0, p.N, kb, ke);
    oa.store(lds);
    ob.store(lds + OA::LDS);
  }
  __syncthreads();
  int cur = 0;
  for (int k0 = kb; k0 < ke; k0 += BK) {
    const bool more = k0 + BK < ke;
    if (more) {
      oa.load(p, p.A, p.lda, m0, p.M, k0 + BK, ke);
      ob.load(p, p.B, p.ldb, n0, p.N, k0 + BK, ke);
    }
    const float* As = lds + cur * STAGE;
    const float* Bs = As + OA::LDS;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      float4 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = oa.frag(As, wm * WM + i * 32 + lr, g, lh);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = ob.frag(Bs, wn * WN + j * 32 + lr, g, lh);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(fa[i], s), f4get(fb[j], s), acc[i][j], 0, 0, 0);
    }
    if (more) {
      oa.store(lds + (cur ^ 1) * STAGE);
      ob.store(lds + (cur ^ 1) * STAGE + OA::LDS);
    }
    __syncthreads();
    cur ^= 1;
  }

  // C/D map of the 32x32 f32 MFMA: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  if (!p.atomic) {
    // each wave stages its 32-row slabs through its own LDS region (the k-loop's stages are free
    // after the last barrier) and stores 16 B per lane: WN/4 lanes cover a row segment.
    // With p.stats every lane also accumulates its 4 columns' sum / sum of squares over the rows
    // it stores (the BN statistics of the output, from the values as stored), reduced across the
    // lanes sharing those columns and across the two waves of the column band below.
    float st_s[4] = {0.f, 0.f, 0.f, 0.f}, st_q[4] = {0.f, 0.f, 0.f, 0.f};
    float* slab = lds + w * 32 * CP;
    constexpr int LPR = WN / 4;          // lanes per staged row
    constexpr int RPI = kWave / LPR;     // rows per wave instruction
    const int cq = lane % LPR;
    const int col = n0 + wn * WN + 4 * cq;
    const bool bnb = p.stats != nullptr && p.bx != nullptr;
    float4 bmean = make_float4(0.f, 0.f, 0.f, 0.f), bsc = bmean, bsh = bmean;
    if (bnb && col + 3 < p.N) {
      bmean = *reinterpret_cast<const float4*>(p.bsave + col);
      if (p.bmask == nullptr && p.brelu) {
        bsc = *reinterpret_cast<const float4*>(p.bsave + 2 * p.N + col);
        bsh = *reinterpret_cast<const float4*>(p.bsave + 3 * p.N + col);
      }
    }
    constexpr int NR = 32 / RPI;  // staged rows per lane per slab
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      // BN-backward epilogue: this slab's x (and mask) loads are issued before the slab is staged,
      // so their latency overlaps the staging instead of serialising the row loop
      float4 xpre[bnb_slots(NR)];
      uint32_t mpre[bnb_slots(NR)];
      if (bnb) {
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          const int row = m0 + wm * WM + i * 32 + lane / LPR + j * RPI;
          xpre[j] = make_float4(0.f, 0.f, 0.f, 0.f);
          mpre[j] = 0xfu;
          if (row < p.M && col + 3 < p.N) {
            const int64_t e = (int64_t)row * p.N + col;  // dense [M][N] BN activation (ldc == N)
            xpre[j] = *reinterpret_cast<const float4*>(p.bx + e);
            if (p.bmask != nullptr) mpre[j] = (uint32_t)(p.bmask[e >> 3] >> (e & 7));
          }
        }
      }
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) slab[((r & 3) + 8 * (r >> 2) + 4 * lh) * CP + j * 32 + lr] = acc[i][j][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        const int rr = lane / LPR + j * RPI;
        const int row = m0 + wm * WM + i * 32 + rr;
        if (row < p.M) {
          const float4 v = *reinterpret_cast<const float4*>(slab + rr * CP + 4 * cq);
          float* dst = p.C + (int64_t)row * p.ldc + col;
          if (bnb) {
            if (col + 3 < p.N) {
              const float4 xv = xpre[j];
              uint32_t mb = mpre[j];
              if (p.bmask == nullptr && p.brelu)  // the forward's ReLU test, recomputed: scale * x + shift > 0
                mb = (fmaf(xv.x, bsc.x, bsh.x) > 0.f ? 1u : 0u) | (fmaf(xv.y, bsc.y, bsh.y) > 0.f ? 2u : 0u) |
                     (fmaf(xv.z, bsc.z, bsh.z) > 0.f ? 4u : 0u) | (fmaf(xv.w, bsc.w, bsh.w) > 0.f ? 8u : 0u);
              const float d0 = (mb & 1u) ? v.x : 0.f, d1 = (mb & 2u) ? v.y : 0.f;
              const float d2 = (mb & 4u) ? v.z : 0.f, d3 = (mb & 8u) ? v.w : 0.f;
              st_s[0] += d0; st_s[1] += d1; st_s[2] += d2; st_s[3] += d3;
              st_q[0] = fmaf(d0, xv.x - bmean.x, st_q[0]); st_q[1] = fmaf(d1, xv.y - bmean.y, st_q[1]);
              st_q[2] = fmaf(d2, xv.z - bmean.z, st_q[2]); st_q[3] = fmaf(d3, xv.w - bmean.w, st_q[3]);
            }
          } else if (p.stats != nullptr) {
            st_s[0] += v.x; st_s[1] += v.y; st_s[2] += v.z; st_s[3] += v.w;
            st_q[0] = fmaf(v.x, v.x, st_q[0]); st_q[1] = fmaf(v.y, v.y, st_q[1]);
            st_q[2] = fmaf(v.z, v.z, st_q[2]); st_q[3] = fmaf(v.w, v.w, st_q[3]);
          }
          if (p.c_vec && col + 3 < p.N) {
            *reinterpret_cast<float4*>(dst) = v;
          } else {
            if (col < p.N) dst[0] = v.x;
            if (col + 1 < p.N) dst[1] = v.y;
            if (col + 2 < p.N) dst[2] = v.z;
            if (col + 3 < p.N) dst[3] = v.w;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (p.stats != nullptr) {
      // lanes l, l + LPR, l + 2 LPR ... hold the same 4 columns: butterfly over the row phases
#pragma unroll
      for (int off = LPR; off < kWave; off <<= 1)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          st_s[j] += __shfl_xor(st_s[j], off, kWave);
          st_q[j] += __shfl_xor(st_q[j], off, kWave);
        }
      __syncthreads();  // every wave is done with its slab: reuse the LDS for the wm-pair fold
      float* red = lds;  // [2 (wn)][2 (s, q)][WN]
      if (wm == 1 && lane < LPR) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          red[(wn * 2 + 0) * WN + 4 * cq + j] = st_s[j];
          red[(wn * 2 + 1) * WN + 4 * cq + j] = st_q[j];
        }
      }
      __syncthreads();
      if (wm == 0 && lane < LPR) {
        float* out = p.stats + (int64_t)tm * 2 * p.N;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = col + j;
          if (c < p.N) {
            out[c] = st_s[j] + red[(wn * 2 + 0) * WN + 4 * cq + j];
            out[p.N + c] = st_q[j] + red[(wn * 2 + 1) * WN + 4 * cq + j];
          }
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = n0 + wn * WN + j * 32 + lr;
      if (col >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row < p.M) {
          float* dst = p.C + (int64_t)row * p.ldc + col;
          atomicAdd(dst, acc[i][j][r]);
        }
      }
    }
}

template <int BM, int BN, int AM, int BMD>
int launch_cfg(GemmParams p, hipStream_t stream) {
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.N + BN - 1) / BN;
  const int64_t blocks = (int64_t)p.tiles_m * p.tiles_n * p.splits;
  gemm_f32_kernel<BM, BN, AM, BMD><<<(unsigned)blocks, kGB, 0, stream>>>(p);
  return p.tiles_m;
}

inline int64_t ntiles(int M, int N, int bm, int bn) { return (int64_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn); }

// tile shape: the largest of 128x128 / 128x64 / 64x128 / 64x64 that still gives >= 1.5 workgroups
// per CU (small-M layers, e.g. the 7x7 stage at M = 1568, otherwise leave most of the chip idle)
template <int AM, int BMD>
int launch_layout(GemmParams p, hipStream_t stream) {
  const int64_t want = 384;
  const int64_t t128 = ntiles(p.M, p.N, 128, 128) * p.splits;
  const int64_t tm = ntiles(p.M, p.N, 128, 64) * p.splits, tn = ntiles(p.M, p.N, 64, 128) * p.splits;
  if (p.M > 64 && p.N > 64 && t128 >= want) return launch_cfg<128, 128, AM, BMD>(p, stream);
  if (p.M > 64 && tm >= want && (p.N <= 64 || tm >= tn)) return launch_cfg<128, 64, AM, BMD>(p, stream);
  if (p.N > 64 && tn >= want) return launch_cfg<64, 128, AM, BMD>(p, stream);
  return launch_cfg<64, 64, AM, BMD>(p, stream);
}

}  // namespace

namespace {
// tile: 0 = by the launcher's rule, 1 = 128x128, 2 = 128x64, 3 = 64x128, 4 = 64x64 (the bindings
// reject anything else)
template <int AM, int BMD>
int launch_tile(GemmParams p, int tile, hipStream_t stream) {
  switch (tile) {
    case 1: return launch_cfg<128, 128, AM, BMD>(p, stream);
    case 2: return launch_cfg<128, 64, AM, BMD>(p, stream);
    case 3: return launch_cfg<64, 128, AM, BMD>(p, stream);
    case 4: return launch_cfg<64, 64, AM, BMD>(p, stream);
    default: return launch_layout<AM, BMD>(p, stream);
  }
}

// split-K rule shared by the plain and the implicit GEMMs: split K when even 64x64 tiles leave
// CUs idle (f32 atomics into a zeroed, dense C)
int auto_splits(int M, int N, int K, int64_t ldc) {
  const int64_t tiles = ntiles(M, N, 64, 64);
  int splits = 1;
  if (tiles < 256 && K >= 512 && ldc == N) splits = (int)std::min<int64_t>((384 + tiles - 1) / tiles, K / 256);
  return splits;
}

// splits -> k per split (multiple of BK), C zeroed for split-K; returns whether atomic
void set_splits(GemmParams& p, int splits, float* stats, hipStream_t stream) {
  if (splits < 1) splits = 1;
  int kps = (p.K + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  splits = p.K > 0 ? (p.K + kps - 1) / kps : 1;
  p.splits = splits;
  p.k_per_split = kps;
  p.atomic = splits > 1;
  p.c_vec = (reinterpret_cast<uintptr_t>(p.C) % 16 == 0) && (p.ldc % 4 == 0);
  p.stats = p.atomic ? nullptr : stats;  // statistics need whole-K tiles (the binding checks)
  if (p.atomic) GRACE_HIP_CHECK(hipMemsetAsync(p.C, 0, sizeof(float) * (size_t)p.M * p.ldc, stream));  // ldc == N
}
}  // namespace

int gemm_f32(const float* A, bool a_kcontig, int64_t lda, const float* B, bool b_kcontig, int64_t ldb, float* C,
             int64_t ldc, int M, int N, int K, int splits, hipStream_t stream, int tile, float* stats,
             const BnBwdEpi* bnb, const BnApplyPro* xf) {
  if (M <= 0 || N <= 0) return 0;
  GemmParams p{};
  if (bnb != nullptr) {
    p.bx = bnb->x;
    p.bmask = bnb->mask;
    p.bsave = bnb->save;
    p.brelu = bnb->relu;
  }
  if (xf != nullptr) {
    p.xsave = xf->save;
    p.xC = xf->C;
    p.xrelu = xf->relu;
    p.xop = xf->op;
  }
  p.A = A;
  p.B = B;
  p.C = C;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = ldb;
  p.ldc = ldc;
  if (splits == 0) splits = auto_splits(M, N, K, ldc);  // host-checked: split-K only with ldc == N
  set_splits(p, splits, stats, stream);
  if (a_kcontig && b_kcontig) return launch_tile<0, 0>(p, tile, stream);
  if (a_kcontig && !b_kcontig) return launch_tile<0, 1>(p, tile, stream);
  if (!a_kcontig && !b_kcontig) return launch_tile<1, 1>(p, tile, stream);
  return launch_tile<1, 0>(p, tile, stream);
}

int conv3x3_f32(int dir, const float* act, const float* other, float* C, int N, int H, int W, int Cin, int Cout,
                int stride, int splits, int tile, float* stats, hipStream_t stream, int ksize, const BnBwdEpi* bnb,
                const BnApplyPro* xf) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;  // 3x3 pad 1, or 1x1 pad 0
  const int T = ksize * ksize;
  GemmParams p{};
  if (bnb != nullptr && dir == 1) {
    p.bx = bnb->x;
    p.bmask = bnb->mask;
    p.bsave = bnb->save;
    p.brelu = bnb->relu;
  }
  if (xf != nullptr && dir != 1) {  // the activation operand: A of the forward, B of the weight grad
    p.xsave = xf->save;
    p.xC = xf->C;
    p.xrelu = xf->relu;
    p.xop = dir == 0 ? 1 : 2;
  }
  p.C = C;
  if (dir == 0) {  // forward: rows = output pixels, k = (tap, ci)
    p.A = act;
    p.B = other;
    p.M = N * Ho * Wo;
    p.N = Cout;
    p.K = T * Cin;
    p.ldb = T * Cin;
    p.ldc = Cout;
    p.gHr = Ho, p.gWr = Wo, p.gHs = H, p.gWs = W, p.gC = Cin, p.gS = stride, p.gSign = 1;
  } else if (dir == 1) {  // data grad (stride 1): rows = input pixels, k = (tap, co), flipped taps
    p.A = act;  // dY [N, H, W, Cout]
    p.B = other;
    p.M = N * H * W;
    p.N = Cin;
    p.K = T * Cout;
    p.ldb = T * Cin;
    p.ldc = Cin;
    p.kt = Cout;
    p.tap_off = Cin;
    p.gHr = H, p.gWr = W, p.gHs = H, p.gWs = W, p.gC = Cout, p.gS = 1, p.gSign = -1;
  } else {  // weight grad: [Cout][(tap, ci)] over k = output pixels
    p.A = other;  // dY [N, Ho, Wo, Cout]: MN-contig, ld = Cout
    p.B = act;    // x
    p.M = Cout;
    p.N = T * Cin;
    p.K = N * Ho * Wo;
    p.lda = Cout;
    p.ldc = T * Cin;
    p.gHr = Ho, p.gWr = Wo, p.gHs = H, p.gWs = W, p.gC = Cin, p.gS = stride, p.gSign = 1;
  }
  p.gT = ksize;
  p.gInvWr = 1.f / (float)p.gWr;
  p.gInvHr = 1.f / (float)p.gHr;
  if (p.M <= 0 || p.N <= 0) return 0;
  if (splits == 0) splits = dir == 2 ? auto_splits(p.M, p.N, p.K, p.ldc) : 1;
  set_splits(p, splits, (dir == 0 || p.bx != nullptr) ? stats : nullptr, stream);
  if (dir == 0) return launch_tile<2, 0>(p, tile, stream);
  if (dir == 1) return launch_tile<2, 4>(p, tile, stream);
  return launch_tile<1, 3>(p, tile, stream);
}

}  // namespace grace
