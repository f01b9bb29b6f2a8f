// swarm_policy.hip — on-device actor inference for the swarm rollout loop (gfx950, MFMA).
//
// The reference's actor is RLlib's TorchFC with fcnet_hiddens [256, 256] and relu
// (src/swarm_marl/training/config_builders.py:53-56, models.py:75-81), exported by
// scripts/export_onnx.py:120-141 as  logits = Gemm(Relu(Gemm(Relu(Gemm(obs)))))  (transB = 1).
// RLlib's TorchDiagGaussian reads logits = [mean | log_std]; its deterministic action is the mean.
//
// swarm_policy_forward runs that MLP over `rows` observation rows (E x N agents of a VecSwarm,
// obs [E,N,D] read in place) and writes logits and/or actions [rows, out/2] (the env's action
// tensor), so observations never leave HBM between env steps.
//
// bf16 path (default): v_mfma_f32_32x32x16_bf16, f32 accumulation.  One wave owns a tile of 32
// obs rows and computes every layer TRANSPOSED, C[out][row] = W · X^T: the row index sits on
// the lane, so a layer's f32 accumulators, relu'd and packed to bf16 in place, ARE the next
// layer's B operand (no LDS round trip, no shuffles).  The k order of such an operand is the
// accumulator's register order (element j of lane half h in k-step s is row
// 16s + 8(j>>2) + 4h + (j&3) of the 32-row block), so the host packs W2 / W3 with that
// permutation of their input index.  Weights live in LDS in MFMA-fragment order (one 1-KB block
// of 64 lanes x 16 B per (out block, k step): every A read is one conflict-free ds_read_b128);
// the layer-1 bias rides in the pad column k = D of the obs fragment (x[D] = 1).
// f32 path: v_mfma_f32_16x16x4_f32 (f32 products, f32 sums: within summation-order rounding of
// the f32 graph) on 16-row tiles, the same accumulator-as-operand chaining; A fragments stream
// from global memory (L2-resident, 256 B per wave-instruction).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "swarm_mi355x.h"

#pragma clang fp contract(off)

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int H = SWARM_POLICY_HIDDEN;  // 256
constexpr int KP1 = 48;                 // bf16 layer-1 K (obs dim + bias column, padded)
constexpr int KS1 = KP1 / 16;           // 3 k-steps
constexpr int OB = H / 32;              // 8 out blocks of 32 (bf16 path)
constexpr int KS2 = H / 16;             // 16 k-steps over the hidden dim
constexpr int FRAG = 1024;              // bytes of one 64-lane x 16-B fragment block

// ---------------------------------------------------------------- packed blob layouts
// bf16: [W1F 8x3 blocks][W2F 8x16 blocks][W3F 16 k-steps x 2*out lanes x 16 B][b2 256 f32][b3 32 f32]
struct Bf16Layout {
  int out;
  size_t w1, w2, w3, b2, b3, total;
  __host__ __device__ explicit Bf16Layout(int o) : out(o) {
    w1 = 0;
    w2 = w1 + (size_t)OB * KS1 * FRAG;
    w3 = w2 + (size_t)OB * KS2 * FRAG;
    b2 = w3 + (size_t)KS2 * 2 * o * 16;
    b3 = b2 + H * 4;
    total = b3 + 32 * 4;
  }
};
// f32: [W1 16 obs x KQ1 q x 64 lanes][W2 16 x 64 x 64][W3 64 x 64][b2 256][b3 16] floats
struct F32Layout {
  int kq1;
  size_t w1, w2, w3, b2, b3, total;  // float offsets
  __host__ __device__ explicit F32Layout(int in) {
    kq1 = (in + 1 + 3) / 4;
    w1 = 0;
    w2 = w1 + (size_t)16 * kq1 * 64;
    w3 = w2 + (size_t)16 * 64 * 64;
    b2 = w3 + (size_t)64 * 64;
    b3 = b2 + H;
    total = b3 + 16;
  }
};

// hidden unit carried by k-step `ks` (of 16) of an accumulator-chained operand, lane half h, element j
__host__ __device__ inline int chained_k(int ks, int h, int j) {
  return (ks >> 1) * 32 + 16 * (ks & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
}
// f32 16x16x4 chaining: k-step q (of 64) of lane quarter g -> hidden unit
__host__ __device__ inline int chained_k_f32(int q, int g) { return (q >> 2) * 16 + 4 * g + (q & 3); }

// IEEE binary16, round to nearest even (subnormals kept; overflow -> inf); and back
uint16_t f16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  const uint32_t sign = (u >> 16) & 0x8000u;
  const uint32_t a = u & 0x7fffffffu;
  if (a >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0u));
  if (a >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds past 65504
  if (a < 0x38800000u) {  // f16 subnormal (or zero): value / 2^-24, rounded to nearest even
    if (a < 0x33000000u) return (uint16_t)sign;  // below half the smallest subnormal
    const uint32_t e = a >> 23, mant = (a & 0x7fffffu) | 0x800000u;
    const int shift = 126 - (int)e;  // mant * 2^(e-150) / 2^-24 = mant >> (126 - e)
    uint32_t q = mant >> shift;
    const uint32_t rem = mant & ((1u << shift) - 1u), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (q & 1u))) ++q;
    return (uint16_t)(sign | q);
  }
  uint32_t r = a - 0x38000000u;  // rebias 127 -> 15
  const uint32_t lsb = (r >> 13) & 1u;
  r += 0xfffu + lsb;
  return (uint16_t)(sign | (r >> 13));
}
float f16_to_f32(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  float f;
  if (e == 0) {
    f = (float)m * 0x1p-24f;
    return sign ? -f : f;
  }
  uint32_t u = e == 31 ? (sign | 0x7f800000u | (m << 13)) : (sign | ((e + 112u) << 23) | (m << 13));
  memcpy(&f, &u, 4);
  return f;
}

uint16_t bf16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// ---------------------------------------------------------------- bf16 kernel
__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }

// 8 accumulator values -> bf16 fragment, relu'd after the conversion: round-to-nearest keeps the
// sign, so relu(bf16(x)) == bf16(relu(x)), and a bf16 with the sign bit set is a negative int16:
// one v_pk_max_i16 with 0 relus two values (an f32 relu costs a canonicalising v_max plus the max
// on MFMA outputs: 4x the instructions).
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) short s16x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
__device__ __forceinline__ bf16x8 pack8(const f32x16& a, int s, bool act) {
  u32x4 w;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const bf16x2 p = __builtin_convertvector((f32x2){a[8 * s + 2 * q], a[8 * s + 2 * q + 1]}, bf16x2);  // v_cvt_pk_bf16_f32
    s16x2 v = __builtin_bit_cast(s16x2, p);
    if (act) v = __builtin_elementwise_max(v, (s16x2){0, 0});  // v_pk_max_i16
    w[q] = __builtin_bit_cast(unsigned, v);
  }
  return __builtin_bit_cast(bf16x8, w);
}

// Philox4x32-10 (same constants as the env's device reset)
__device__ __forceinline__ void philox(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

struct FwdArgs {
  const void* w;        // packed blob (device)
  const float* obs;     // [rows, in]
  float* logits;        // [rows, out] or null
  float* actions;       // [rows, out/2] or null
  long long rows;
  int in, out, mode;    // mode: 0 mean, 1 sample
  uint32_t seed_lo, seed_hi, ctr_lo, ctr_hi;
};

// T row tiles per wave (T = 2: every weight fragment read from LDS feeds two MFMAs, halving the
// LDS bytes per FLOP — one 1-KB A fragment per 32x32x16 MFMA is the whole LDS bandwidth of a CU
// at the MFMA peak; T = 2 needs ~330 registers, i.e. one wave per SIMD).
// IN_C / OUT_C: compile-time obs / logits widths (0 = runtime): the obs gather's pad and bias
// selects and the layer-3 row masks fold away for the env's default D = 37, out = 6.
template <int WAVES, int MODE, int T, int IN_C = 0, int OUT_C = 0>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(WAVES / 4 > 0 ? WAVES / 4 : 1)))
policy_mlp_bf16(const FwdArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const Bf16Layout L(A.out);
  {  // stage the packed weights (~159 KB) in LDS, once per workgroup: 8 loads in flight per
     // thread per round (a load-then-store loop pays one global round trip per 16 B x threads)
    const int4* src = reinterpret_cast<const int4*>(A.w);
    int4* dst = reinterpret_cast<int4*>(lds);
    const int n16 = (int)(L.total / 16);
    constexpr int UNR = 8, STRIDE = 64 * WAVES;
    for (int base = threadIdx.x; base < n16; base += STRIDE * UNR) {
      int4 v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int i = base + u * STRIDE;
        v[u] = src[i < n16 ? i : n16 - 1];
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int i = base + u * STRIDE;
        if (i < n16) dst[i] = v[u];
      }
    }
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6;
  const long long ntiles = (A.rows + 31) / 32;
  const long long ngroups = (ntiles + T - 1) / T;
  const float* b2 = reinterpret_cast<const float*>(lds + L.b2);
  const float* b3 = reinterpret_cast<const float*>(lds + L.b3);
  for (long long grp = (long long)blockIdx.x * WAVES + wave; grp < ngroups; grp += (long long)gridDim.x * WAVES) {
    // Opaque per tile group: the lane index and the layer dims.  Everything derived from them
    // (fragment addresses, the obs element offsets and their pad/bias selects, the layer-3 row
    // masks) is recomputed per group instead of being hoisted out of the loop, where it would
    // stay live next to h1/h2 and spill.
    int lane = threadIdx.x & 63, in_r = A.in, out_r = A.out;
    asm volatile("" : "+v"(lane), "+s"(in_r), "+s"(out_r));
    const int in = IN_C ? IN_C : in_r, out = OUT_C ? OUT_C : out_r;
    const int n = lane & 31, h = (lane >> 5) & 1;  // h in [0, 1]: k-range facts fold the obs selects
    const bool w3lane = n < out;
    const int w3idx = h * out + n;
    const uint32_t lb = 16u * (uint32_t)lane;
    const bf16x8* w1f = reinterpret_cast<const bf16x8*>(lds + L.w1 + lb);
    const bf16x8* w2f = reinterpret_cast<const bf16x8*>(lds + L.w2 + lb);
    const bf16x8* w3f = reinterpret_cast<const bf16x8*>(lds + L.w3);
    long long row[T];
    bool valid[T];
#pragma unroll
    for (int u = 0; u < T; ++u) {
      row[u] = (grp * T + u) * 32 + n;
      valid[u] = row[u] < A.rows;
    }
    // ---- obs fragments (B of layer 1): x[row][16 ks + 8 h + j], x[in] = 1 (bias column).
    // Unconditional loads from clamped addresses (one wait for all of them), then selects.
    bf16x8 xb[T][KS1];
#pragma unroll
    for (int u = 0; u < T; ++u) {
      const float* xr = A.obs + (valid[u] ? row[u] : A.rows - 1) * in;
      float xv[KS1 * 8];
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 16 * ks + 8 * h + j;
          xv[ks * 8 + j] = xr[k < in ? k : in - 1];
        }
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 16 * ks + 8 * h + j;
          xb[u][ks][j] = (__bf16)(k < in ? xv[ks * 8 + j] : (k == in ? 1.f : 0.f));
        }
    }
    // ---- layer 1: 256 x (in + 1), relu -> h1 (16 k-step fragments per tile)
    bf16x8 h1[T][KS2];
#pragma unroll
    for (int ob = 0; ob < OB; ++ob) {
      f32x16 acc[T];
#pragma unroll
      for (int u = 0; u < T; ++u) acc[u] = f32x16{};
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
        const bf16x8 w = w1f[(ob * KS1 + ks) * 64];
#pragma unroll
        for (int u = 0; u < T; ++u) acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w, xb[u][ks], acc[u], 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < T; ++u) {
        h1[u][2 * ob] = pack8(acc[u], 0, true);
        h1[u][2 * ob + 1] = pack8(acc[u], 1, true);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep each out block's fragment reads inside it
    }
    // ---- layer 2 (256 x 256, relu) fused with layer 3 (out x 256): each out block's two
    // relu'd bf16 fragments are the B operands of layer 3's k-steps 2ob, 2ob+1 right away, so h2
    // is never held whole (64 fewer VGPRs per tile)
    f32x16 acc3[T];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = (i & 3) + 8 * (i >> 2) + 4 * h;
#pragma unroll
      for (int u = 0; u < T; ++u) acc3[u][i] = m < out ? b3[m] : 0.f;
    }
#pragma unroll
    for (int ob = 0; ob < OB; ++ob) {
      f32x16 acc[T];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 b = *reinterpret_cast<const float4*>(b2 + ob * 32 + 8 * g + 4 * h);
#pragma unroll
        for (int u = 0; u < T; ++u) {
          acc[u][4 * g + 0] = b.x; acc[u][4 * g + 1] = b.y; acc[u][4 * g + 2] = b.z; acc[u][4 * g + 3] = b.w;
        }
      }
#pragma unroll
      for (int ks = 0; ks < KS2; ++ks) {
        const bf16x8 w = w2f[(ob * KS2 + ks) * 64];
#pragma unroll
        for (int u = 0; u < T; ++u) acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w, h1[u][ks], acc[u], 0, 0, 0);
        if ((ks & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // <= 8 fragments (32 VGPRs) in flight
      }
      bf16x8 a0 = {}, a1 = {};
      if (w3lane) {
        a0 = w3f[(2 * ob) * 2 * out + w3idx];
        a1 = w3f[(2 * ob + 1) * 2 * out + w3idx];
      }
#pragma unroll
      for (int u = 0; u < T; ++u) {
        acc3[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, pack8(acc[u], 0, true), acc3[u], 0, 0, 0);
        acc3[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, pack8(acc[u], 1, true), acc3[u], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int u = 0; u < T; ++u) {
      // ---- outputs: lane holds logits m = (i&3) + 8(i>>2) + 4h of its row (out <= 12: i < 8)
      if (A.logits && valid[u]) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = (i & 3) + 8 * (i >> 2) + 4 * h;
          if (m < out) A.logits[row[u] * out + m] = acc3[u][i];
        }
      }
      if (A.actions) {
        // gather the row's logits 0..11 on the writing lane (half h = 0): it holds m 0-3 and
        // 8-11, its partner n + 32 holds m 4-7 (static indices: no per-element selects)
        float lg[12];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          lg[i] = acc3[u][i];
          lg[4 + i] = __shfl_xor(acc3[u][i], 32);
          lg[8 + i] = acc3[u][4 + i];
        }
        const int ad = out / 2;
        if (h == 0 && valid[u]) {
          float z[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          if constexpr (MODE == SWARM_POLICY_ACT_SAMPLE) {  // Box-Muller normals from Philox(seed; row, counter)
            const long long r = row[u];
            uint32_t c[4] = {(uint32_t)r, (uint32_t)((unsigned long long)r >> 32), A.ctr_lo, A.ctr_hi};
            philox(c, A.seed_lo, A.seed_hi);
            uint32_t c2[4] = {(uint32_t)r, (uint32_t)((unsigned long long)r >> 32) ^ 0x80000000u, A.ctr_lo, A.ctr_hi};
            if (ad > 2) philox(c2, A.seed_lo, A.seed_hi);
            const uint32_t uu[8] = {c[0], c[1], c[2], c[3], c2[0], c2[1], c2[2], c2[3]};
#pragma unroll
            for (int p = 0; p < 3; ++p) {
              const float u1 = ((float)(uu[2 * p] >> 8) + 0.5f) * 0x1p-24f;
              const float u2 = (float)(uu[2 * p + 1] >> 8) * 0x1p-24f;
              const float rr = sqrtf(-2.f * logf(u1));
              z[2 * p] = rr * cosf(6.28318530717958647692f * u2);
              z[2 * p + 1] = rr * sinf(6.28318530717958647692f * u2);
            }
          }
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            if (k < ad) {
              float a = lg[k];
              if constexpr (MODE == SWARM_POLICY_ACT_SAMPLE) a = a + expf(lg[ad + k]) * z[k];
              A.actions[row[u] * ad + k] = a;
            }
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------- f32 kernel (16-row tiles)
// A fragments are read with buffer loads: one lane-offset VGPR for every load of a tile, the
// fragment's byte offset in an SGPR (per-lane 64-bit addresses for ~1,200 distinct fragments
// would be hoisted out of the tile loop and spilled).
constexpr int BUF_DWORD3 = 0x00020000;  // gfx9 raw buffer descriptor word 3
__device__ __forceinline__ float wload(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t sbase, uint32_t soff_floats) {
  return __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)(sbase + soff_floats * 4u), 0));
}

template <int WAVES>
__global__ void __launch_bounds__(64 * WAVES) policy_mlp_f32(const FwdArgs A) {
  const F32Layout L(A.in);
  const __amdgpu_buffer_rsrc_t W =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(A.w), 0, (int)(L.total * 4), BUF_DWORD3);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const long long ntiles = (A.rows + 15) / 16;
  const int in = A.in, out = A.out, kq1 = L.kq1;
  for (long long tile = (long long)blockIdx.x * WAVES + wave; tile < ntiles; tile += (long long)gridDim.x * WAVES) {
    uint32_t voff = 4u * (uint32_t)lane, sb = 0;
    // opaque per tile: neither the lane offset nor the ~1,200 fragment offsets (SGPR soffset =
    // sb + constant) are hoisted out of the tile loop, where they would be live and spill
    asm volatile("" : "+v"(voff), "+s"(sb));
    const long long row = tile * 16 + n;
    const bool valid = row < A.rows;
    const float* xr = A.obs + (valid ? row : 0) * in;
    // ---- layer 1
    f32x4 h1[16];
#pragma unroll
    for (int ob = 0; ob < 16; ++ob) h1[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < kq1; ++q) {
      const int k = 4 * q + g;
      const float x = k < in ? (valid ? xr[k] : 0.f) : (k == in ? 1.f : 0.f);
#pragma unroll
      for (int ob = 0; ob < 16; ++ob)
        h1[ob] = __builtin_amdgcn_mfma_f32_16x16x4f32(wload(W, voff, sb, (uint32_t)(L.w1 + ((size_t)ob * kq1 + q) * 64)), x,
                                                      h1[ob], 0, 0, 0);
    }
#pragma unroll
    for (int ob = 0; ob < 16; ++ob)
#pragma unroll
      for (int i = 0; i < 4; ++i) h1[ob][i] = relu(h1[ob][i]);
    // ---- layer 2
    f32x4 h2[16];
#pragma unroll
    for (int ob = 0; ob < 16; ++ob) {
      f32x4 acc;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = wload(W, 4u * (uint32_t)(4 * g + i), sb, (uint32_t)(L.b2 + ob * 16));
#pragma unroll
      for (int q = 0; q < 64; ++q) {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wload(W, voff, sb, (uint32_t)(L.w2 + ((size_t)ob * 64 + q) * 64)),
                                                   h1[q >> 2][q & 3], acc, 0, 0, 0);
        if ((q & 15) == 15) __builtin_amdgcn_sched_barrier(0);  // at most 16 fragment loads in flight
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = relu(acc[i]);
      h2[ob] = acc;
    }
    // ---- layer 3 (out <= 16)
    f32x4 acc;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (4 * g + i) < out ? wload(W, 4u * (uint32_t)(4 * g + i), sb, (uint32_t)L.b3) : 0.f;
#pragma unroll
    for (int q = 0; q < 64; ++q) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wload(W, voff, sb, (uint32_t)(L.w3 + (size_t)q * 64)), h2[q >> 2][q & 3],
                                                 acc, 0, 0, 0);
      if ((q & 15) == 15) __builtin_amdgcn_sched_barrier(0);
    }
    // lane holds logits m = 4g + i of its row
    if (A.logits && valid) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (4 * g + i < out) A.logits[row * out + 4 * g + i] = acc[i];
    }
    if (A.actions && valid) {
      const int ad = out / 2;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (4 * g + i < ad) A.actions[row * ad + 4 * g + i] = acc[i];
    }
  }
}

// ---------------------------------------------------------------- f32x3 kernel (split f16, three passes)
// The f32 graph at f16-MFMA speed (SWARM_POLICY_F32X3): every f32 operand v is split into
// hi = f16(v) and lo = f16((v - hi) * 2^11) (v - hi is exact in f32 and at most half an f16 ulp,
// 2^-11 |v|, so the scaled lo stays in the f16 normal range down to |v| ~ 6e-5 and keeps 11
// bits: |v - hi - lo 2^-11| <= 2^-22 |v|).  Every product is hi*hi into one f32 accumulator and
// hi*lo + lo*hi into a second (both scaled by 2^11) on v_mfma_f32_32x32x16_f16; the layer output
// is acc_hh + 2^-11 acc_x.  The dropped lo*lo term is <= 2^-22 relative, so each product carries
// ~2^-21 relative error against f32's 2^-24 and the layer sums stay within the f32 path's
// tolerance.  (Unscaled, lo of a weight below ~0.1 is an f16 subnormal and loses bits.)
// Structure of policy_mlp_bf16 (T = 1): transposed layers, accumulators split in place into the
// next layer's hi / lo B fragments; W hi in LDS (the bf16 blob's fragment order, f16 elements),
// W lo streamed from global memory (L1 / L2-resident: every wave of a workgroup reads the same
// fragments in the same order) by buffer loads with SGPR offsets.
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr float X3_LO_SCALE = 2048.f, X3_LO_INV = 1.f / 2048.f;
constexpr int X3_B = 8;      // W2 k-steps per lo-fragment batch (divides 16; 4 measured slower, r05k)
constexpr int X3_DEPTH = 2;  // W2 lo batches in flight (3 / 4 measured no faster, r05k)
// Tried and measured slower or equal: three accumulator chains (hi*lo and
// lo*hi apart), layer-3 lo fragments requested a block early, W1 / W3 lo fragments a block ahead,
// the next tile's observations prefetched into registers (spills) or touched into L2, and the
// out-block epilogues software-pipelined into the next block's MFMAs with sched_group_barrier.

// 8 accumulator values (sub-block s) -> hi / lo f16 fragments, relu'd first when `act`
__device__ __forceinline__ void split8(const f32x16& a, int s, bool act, f16x8& hi, f16x8& lo) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float x0 = a[8 * s + 2 * q], x1 = a[8 * s + 2 * q + 1];
    if (act) {
      x0 = x0 > 0.f ? x0 : 0.f;
      x1 = x1 > 0.f ? x1 : 0.f;
    }
    const f16x2 h = __builtin_convertvector((f32x2){x0, x1}, f16x2);
    const f32x2 hb = __builtin_convertvector(h, f32x2);
    const f16x2 l = __builtin_convertvector((f32x2){(x0 - hb.x) * X3_LO_SCALE, (x1 - hb.y) * X3_LO_SCALE}, f16x2);
    hi[2 * q] = h.x; hi[2 * q + 1] = h.y;
    lo[2 * q] = l.x; lo[2 * q + 1] = l.y;
  }
}
// soff is wave-uniform; readfirstlane says so to the compiler, which otherwise may compute it in a
// VGPR and wrap the load in a waterfall loop (policy_mlp_x3l did: 23 loops per tile)
__device__ __forceinline__ f16x8 wlo_load(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                       r, (int)voff, __builtin_amdgcn_readfirstlane((int)soff), 0));
}
// hi*hi into c, both cross terms (scaled by 2^11) into x: a dependent 32x32x16 MFMA issues back to
// back on gfx950 (MI355X_MICROARCH.md: one accumulator chain runs at the full 32 cycles per MFMA),
// so a second cross-term chain buys nothing and costs 16 registers per accumulator set
__device__ __forceinline__ void mfma3(const f16x8& ah, const f16x8& al, const f16x8& bh, const f16x8& bl, f32x16& c,
                                      f32x16& x) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, x, 0, 0, 0);
}
__device__ __forceinline__ f32x16 x3_sum(const f32x16& c, const f32x16& x) {
  f32x16 r;
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = c[i] + x[i] * X3_LO_INV;
  return r;
}

template <int WAVES, int IN_C = 0, int OUT_C = 0>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(WAVES / 4 > 0 ? WAVES / 4 : 1)))
policy_mlp_x3(const FwdArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const Bf16Layout L(A.out);
  {  // stage the hi blob (f16 fragments + f32 biases, ~159 KB) in LDS, once per workgroup
    const int4* src = reinterpret_cast<const int4*>(A.w);
    int4* dst = reinterpret_cast<int4*>(lds);
    const int n16 = (int)(L.total / 16);
    constexpr int UNR = 8, STRIDE = 64 * WAVES;
    for (int base = threadIdx.x; base < n16; base += STRIDE * UNR) {
      int4 v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int i = base + u * STRIDE;
        v[u] = src[i < n16 ? i : n16 - 1];
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int i = base + u * STRIDE;
        if (i < n16) dst[i] = v[u];
      }
    }
  }
  __syncthreads();
  // the lo blob: right after the hi blob
  const __amdgpu_buffer_rsrc_t WL = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(reinterpret_cast<const unsigned char*>(A.w) + L.total), 0, (int)L.total, BUF_DWORD3);
  const int wave = threadIdx.x >> 6;
  const long long ntiles = (A.rows + 31) / 32;
  const float* b2 = reinterpret_cast<const float*>(lds + L.b2);
  const float* b3 = reinterpret_cast<const float*>(lds + L.b3);
  // The next tile's observations, requested in the tail of the current tile (after its last
  // layer-2 MFMAs, when h1 is dead) so that the next tile starts on landed data: one wave per SIMD
  // has nothing else to hide that load's latency with (~26 us of 262 without it, r05ai).  The index
  // is clamped rather than branched on, so the values are redefined on every path and dead
  // between their use and the refill.
  float xvn[KS1 * 8];
  auto request_obs = [&](long long tl, int n_, int h_, int in_) {
    const long long r = tl * 32 + n_;
    const float* xr = A.obs + (r < A.rows ? r : A.rows - 1) * in_;
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * ks + 8 * h_ + j;
        xvn[ks * 8 + j] = xr[k < in_ ? k : in_ - 1];
      }
  };
  {
    const long long t0 = (long long)blockIdx.x * WAVES + wave;
    const int ln = threadIdx.x & 63;
    request_obs(t0 < ntiles ? t0 : 0, ln & 31, (ln >> 5) & 1, IN_C ? IN_C : A.in);
  }
  for (long long tile = (long long)blockIdx.x * WAVES + wave; tile < ntiles; tile += (long long)gridDim.x * WAVES) {
    int lane = threadIdx.x & 63, in_r = A.in, out_r = A.out;
    uint32_t sb = 0;
    asm volatile("" : "+v"(lane), "+s"(in_r), "+s"(out_r), "+s"(sb));
    const int in = IN_C ? IN_C : in_r, out = OUT_C ? OUT_C : out_r;
    const int n = lane & 31, h = (lane >> 5) & 1;
    const bool w3lane = n < out;
    const int w3idx = h * out + n;
    const uint32_t lb = 16u * (uint32_t)lane;
    const f16x8* w1f = reinterpret_cast<const f16x8*>(lds + L.w1 + lb);
    const f16x8* w2f = reinterpret_cast<const f16x8*>(lds + L.w2 + lb);
    const f16x8* w3f = reinterpret_cast<const f16x8*>(lds + L.w3);
    const long long row = tile * 32 + n;
    const bool valid = row < A.rows;
    // ---- obs fragments, split: x[row][16 ks + 8 h + j], x[in] = 1 (bias column)
    f16x8 xh[KS1], xl[KS1];
    {
      (void)valid;
      float xv[KS1 * 8];
#pragma unroll
      for (int i = 0; i < KS1 * 8; ++i) xv[i] = xvn[i];
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const int k0 = 16 * ks + 8 * h + j, k1 = k0 + 1;
          const float x0 = k0 < in ? xv[ks * 8 + j] : (k0 == in ? 1.f : 0.f);
          const float x1 = k1 < in ? xv[ks * 8 + j + 1] : (k1 == in ? 1.f : 0.f);
          const f16x2 hh = __builtin_convertvector((f32x2){x0, x1}, f16x2);
          const f32x2 hb = __builtin_convertvector(hh, f32x2);
          const f16x2 ll = __builtin_convertvector((f32x2){(x0 - hb.x) * X3_LO_SCALE, (x1 - hb.y) * X3_LO_SCALE}, f16x2);
          xh[ks][j] = hh.x; xh[ks][j + 1] = hh.y;
          xl[ks][j] = ll.x; xl[ks][j + 1] = ll.y;
        }
    }
    // ---- layer 1: 256 x (in + 1), relu -> h1 hi / lo (16 k-step fragments each)
    // software pipelined like layer 2 below: block ob - 1's epilogue (x3_sum, relu + split into
    // two h1 k-step fragments) interleaved with block ob's nine MFMAs
    f16x8 h1h[KS2], h1l[KS2];
    f32x16 l1acc[2], l1accx[2];
    auto epi1 = [&](int pob, int part) {
      if (part == 0) l1acc[pob & 1] = x3_sum(l1acc[pob & 1], l1accx[pob & 1]);
      else {
        split8(l1acc[pob & 1], part - 1, true, h1h[2 * pob + part - 1], h1l[2 * pob + part - 1]);
        // h1 lo lives in AGPRs (MFMA B operands may come from AGPRs): 64 architectural VGPRs
        // freed for the observation request above (without it the kernel sits at the 256-VGPR cap
        // and that request spills, r05aj)
        asm volatile("" : "+a"(h1l[2 * pob + part - 1]));
      }
    };
#pragma unroll
    for (int ob = 0; ob < OB; ++ob) {
      f32x16& acc = l1acc[ob & 1];
      f32x16& accx = l1accx[ob & 1];
      acc = f32x16{};
      accx = f32x16{};
      f16x8 w1l[KS1];
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) w1l[ks] = wlo_load(WL, lb, sb + (uint32_t)(L.w1 + (size_t)(ob * KS1 + ks) * FRAG));
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
        mfma3(w1f[(ob * KS1 + ks) * 64], w1l[ks], xh[ks], xl[ks], acc, accx);
        if (ob > 0) epi1(ob - 1, ks);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    epi1(OB - 1, 0);
    epi1(OB - 1, 1);
    epi1(OB - 1, 2);
    // ---- layer 2 (relu) fused with layer 3: each out block's two split fragments feed layer 3's
    // k-steps 2ob, 2ob+1 at once
    f32x16 acc3, acc3x = f32x16{};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = (i & 3) + 8 * (i >> 2) + 4 * h;
      acc3[i] = m < out ? b3[m] : 0.f;
    }
    // W2 lo fragments stream in batches of X3_B k-steps, double-buffered: batch b + 1's loads are
    // issued before batch b's MFMAs (128 fragments per wave in (ob, ks) order)
    constexpr int NB2 = OB * KS2 / X3_B;
    constexpr int DEP = X3_DEPTH;  // batches in flight: batch b + DEP - 1 is requested before batch b's MFMAs
    f16x8 wlb[DEP][X3_B];
#pragma unroll
    for (int b0 = 0; b0 + 1 < DEP; ++b0)
#pragma unroll
      for (int u = 0; u < X3_B; ++u) wlb[b0][u] = wlo_load(WL, lb, sb + (uint32_t)(L.w2 + (size_t)(b0 * X3_B + u) * FRAG));
    // Software pipeline over the out blocks: block ob's layer-2 MFMAs accumulate into one of two
    // accumulator pairs while the epilogue of block ob - 1 (x3_sum, relu + hi / lo split, its two
    // layer-3 k-steps) is interleaved with block ob's first batch — at one wave per SIMD nothing
    // else would fill the MFMA pipe during that vector work.
    f32x16 acc2[2], accx2[2];
    f32x16 pacc;           // block ob - 1's layer-2 output
    f16x8 a0h = {}, a1h = {}, a0l = {}, a1l = {};
    auto epi = [&](int pob, int part) {  // a third of block pob's epilogue
      if (part == 0) {
        pacc = x3_sum(acc2[pob & 1], accx2[pob & 1]);
        if (w3lane) {  // this block's layer-3 fragments (k-steps 2pob, 2pob+1), the lo halves from L2
          a0h = w3f[(2 * pob) * 2 * out + w3idx];
          a1h = w3f[(2 * pob + 1) * 2 * out + w3idx];
          a0l = wlo_load(WL, 16u * (uint32_t)w3idx, sb + (uint32_t)(L.w3 + (size_t)(2 * pob) * 2 * out * 16));
          a1l = wlo_load(WL, 16u * (uint32_t)w3idx, sb + (uint32_t)(L.w3 + (size_t)(2 * pob + 1) * 2 * out * 16));
        }
      } else {
        f16x8 h2h, h2l;
        split8(pacc, part - 1, true, h2h, h2l);
        if (part == 1) mfma3(a0h, a0l, h2h, h2l, acc3, acc3x);
        else mfma3(a1h, a1l, h2h, h2l, acc3, acc3x);
      }
    };
#pragma unroll
    for (int ob = 0; ob < OB; ++ob) {
      f32x16& acc = acc2[ob & 1];
      f32x16& accx = accx2[ob & 1];
      accx = f32x16{};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 b = *reinterpret_cast<const float4*>(b2 + ob * 32 + 8 * g + 4 * h);
        acc[4 * g + 0] = b.x; acc[4 * g + 1] = b.y; acc[4 * g + 2] = b.z; acc[4 * g + 3] = b.w;
      }
#pragma unroll
      for (int kb = 0; kb < KS2; kb += X3_B) {
        const int bi = (ob * KS2 + kb) / X3_B;  // batch index
        const int nb = bi + DEP - 1;  // the batch requested now
        if (nb < NB2) {
#pragma unroll
          for (int u = 0; u < X3_B; ++u)
            wlb[nb % DEP][u] = wlo_load(WL, lb, sb + (uint32_t)(L.w2 + (size_t)(nb * X3_B + u) * FRAG));
        }
        f16x8 wh[X3_B];
#pragma unroll
        for (int u = 0; u < X3_B; ++u) wh[u] = w2f[(ob * KS2 + kb + u) * 64];
#pragma unroll
        for (int u = 0; u < X3_B; ++u) {
          mfma3(wh[u], wlb[bi % DEP][u], h1h[kb + u], h1l[kb + u], acc, accx);
          // the previous block's epilogue, in thirds after k-steps 1, 3 and 5 of the block
          if (ob > 0 && kb + u < 6 && (kb + u) % 2 == 1) epi(ob - 1, (kb + u) / 2);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    {  // h1 is dead: the next tile's observations
      const long long nt = tile + (long long)gridDim.x * WAVES;
      request_obs(nt < ntiles ? nt : tile, n, h, in);
    }
    // the last block's epilogue
    epi(OB - 1, 0);
    epi(OB - 1, 1);
    epi(OB - 1, 2);
    acc3 = x3_sum(acc3, acc3x);
    // ---- outputs: lane holds logits m = (i&3) + 8(i>>2) + 4h of its row (out <= 12: i < 8)
    if (A.logits && valid) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = (i & 3) + 8 * (i >> 2) + 4 * h;
        if (m < out) A.logits[row * out + m] = acc3[i];
      }
    }
    if (A.actions) {
      float lg[12];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        lg[i] = acc3[i];
        lg[4 + i] = __shfl_xor(acc3[i], 32);
        lg[8 + i] = acc3[4 + i];
      }
      const int ad = out / 2;
      if (h == 0 && valid) {
#pragma unroll
        for (int k = 0; k < 6; ++k)
          if (k < ad) A.actions[row * ad + k] = lg[k];
      }
    }
  }
}

// f32x3 at two waves per SIMD (8 per workgroup, <= 256 registers each): policy_mlp_x3's arithmetic
// in the same order — every accumulator sees the same MFMA sequence and the same epilogues, so the
// outputs are bit-identical — without its one-wave latency hiding (epilogues interleaved into the
// next block's MFMAs, double-buffered W2 lo batches, the next tile's observations requested early):
// the SIMD's second wave fills those gaps instead, and the registers they held (~490 -> ~250) buy
// that second wave.  Live across layer 2: h1 hi / lo (128), one layer-2 accumulator pair (32), the
// fused layer-3 pair (32) and one k-step's W hi / lo fragments.
#ifndef X3L_GROUP
#define X3L_GROUP 2  // layer-2 k-steps between scheduling barriers
#endif
#ifndef X3L_HI_AHEAD
#define X3L_HI_AHEAD 1  // W2 hi read from LDS one k-step ahead
#endif
#ifndef X3L_AHEAD
#define X3L_AHEAD 1  // W2 lo fragments in flight ahead of their MFMAs (divides 16; 2 / 4 / 8 no faster, r06u)
#endif
template <int WAVES>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(WAVES / 4 > 0 ? WAVES / 4 : 1)))
policy_mlp_x3l(const FwdArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const Bf16Layout L(A.out);
  {  // stage the hi blob in LDS, once per workgroup (as policy_mlp_x3)
    const int4* src = reinterpret_cast<const int4*>(A.w);
    int4* dst = reinterpret_cast<int4*>(lds);
    const int n16 = (int)(L.total / 16);
    constexpr int UNR = 4, STRIDE = 64 * WAVES;
    for (int base = threadIdx.x; base < n16; base += STRIDE * UNR) {
      int4 v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int i = base + u * STRIDE;
        v[u] = src[i < n16 ? i : n16 - 1];
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int i = base + u * STRIDE;
        if (i < n16) dst[i] = v[u];
      }
    }
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t WL = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(reinterpret_cast<const unsigned char*>(A.w) + L.total), 0, (int)L.total, BUF_DWORD3);
  const int wave = threadIdx.x >> 6;
  const long long ntiles = (A.rows + 31) / 32;
  const float* b2 = reinterpret_cast<const float*>(lds + L.b2);
  const float* b3 = reinterpret_cast<const float*>(lds + L.b3);
  for (long long tile = (long long)blockIdx.x * WAVES + wave; tile < ntiles; tile += (long long)gridDim.x * WAVES) {
    int lane = threadIdx.x & 63, in_r = A.in, out_r = A.out;
    uint32_t sb = 0;
    asm volatile("" : "+v"(lane), "+s"(in_r), "+s"(out_r), "+s"(sb));
    const int in = in_r, out = out_r;
    const int n = lane & 31, h = (lane >> 5) & 1;
    const bool w3lane = n < out;
    const int w3idx = h * out + n;
    const uint32_t lb = 16u * (uint32_t)lane;
    const f16x8* w1f = reinterpret_cast<const f16x8*>(lds + L.w1 + lb);
    const f16x8* w2f = reinterpret_cast<const f16x8*>(lds + L.w2 + lb);
    const f16x8* w3f = reinterpret_cast<const f16x8*>(lds + L.w3);
    const long long row = tile * 32 + n;
    const bool valid = row < A.rows;
    // ---- obs fragments, split: x[row][16 ks + 8 h + j], x[in] = 1 (bias column)
    f16x8 xh[KS1], xl[KS1];
    {
      const float* xr = A.obs + (valid ? row : A.rows - 1) * in;
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const int k0 = 16 * ks + 8 * h + j, k1 = k0 + 1;
          const float v0 = xr[k0 < in ? k0 : in - 1], v1 = xr[k1 < in ? k1 : in - 1];
          const float x0 = k0 < in ? v0 : (k0 == in ? 1.f : 0.f);
          const float x1 = k1 < in ? v1 : (k1 == in ? 1.f : 0.f);
          const f16x2 hh = __builtin_convertvector((f32x2){x0, x1}, f16x2);
          const f32x2 hb = __builtin_convertvector(hh, f32x2);
          const f16x2 ll = __builtin_convertvector((f32x2){(x0 - hb.x) * X3_LO_SCALE, (x1 - hb.y) * X3_LO_SCALE}, f16x2);
          xh[ks][j] = hh.x; xh[ks][j + 1] = hh.y;
          xl[ks][j] = ll.x; xl[ks][j + 1] = ll.y;
        }
    }
    // ---- layer 1: 256 x (in + 1), relu -> h1 hi / lo (two k-step fragments per out block)
    f16x8 h1h[KS2], h1l[KS2];
#pragma unroll
    for (int ob = 0; ob < OB; ++ob) {
      f32x16 acc = f32x16{}, accx = f32x16{};
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
        const f16x8 wl = wlo_load(WL, lb, sb + (uint32_t)(L.w1 + (size_t)(ob * KS1 + ks) * FRAG));
        mfma3(w1f[(ob * KS1 + ks) * 64], wl, xh[ks], xl[ks], acc, accx);
      }
      acc = x3_sum(acc, accx);
      split8(acc, 0, true, h1h[2 * ob], h1l[2 * ob]);
      split8(acc, 1, true, h1h[2 * ob + 1], h1l[2 * ob + 1]);
      // h1 lo in AGPRs (MFMA B operands may come from AGPRs), as in policy_mlp_x3
      asm volatile("" : "+a"(h1l[2 * ob]), "+a"(h1l[2 * ob + 1]));
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- layer 2 (relu) fused with layer 3: each out block's two split fragments feed layer 3's
    // k-steps 2ob, 2ob+1
    f32x16 acc3, acc3x = f32x16{};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = (i & 3) + 8 * (i >> 2) + 4 * h;
      acc3[i] = m < out ? b3[m] : 0.f;
    }
    // W2 lo fragments stream X3L_AHEAD k-steps ahead of their MFMAs, across out-block boundaries
    // (fragment q = ob * 16 + ks of the 128; the requests past the last one re-read it)
    f16x8 wlq[X3L_AHEAD];
#pragma unroll
    for (int j = 0; j < X3L_AHEAD; ++j) wlq[j] = wlo_load(WL, lb, sb + (uint32_t)(L.w2 + (size_t)j * FRAG));
#pragma unroll 1
    for (int ob = 0; ob < OB; ++ob) {
      f32x16 acc, accx = f32x16{};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 b = *reinterpret_cast<const float4*>(b2 + ob * 32 + 8 * g + 4 * h);
        acc[4 * g + 0] = b.x; acc[4 * g + 1] = b.y; acc[4 * g + 2] = b.z; acc[4 * g + 3] = b.w;
      }
#if X3L_HI_AHEAD
      f16x8 whq = w2f[(ob * KS2) * 64];  // W2 hi one k-step ahead of its MFMAs (LDS latency)
#endif
#pragma unroll
      for (int ks = 0; ks < KS2; ++ks) {
#if X3L_HI_AHEAD
        const f16x8 wh = whq;
        if (ks + 1 < KS2) whq = w2f[(ob * KS2 + ks + 1) * 64];
#else
        const f16x8 wh = w2f[(ob * KS2 + ks) * 64];
#endif
#ifdef X3L_DIAG_NOWLO  // diagnostic build only (wrong logits): W2 lo from the hi blob in LDS, no W2 lo stream
        const f16x8 wl = w2f[(ob * KS2 + (ks ^ 1)) * 64];
#else
        const f16x8 wl = wlq[ks % X3L_AHEAD];
        const int q = ob * KS2 + ks + X3L_AHEAD;
        wlq[ks % X3L_AHEAD] = wlo_load(WL, lb, sb + (uint32_t)(L.w2 + (size_t)(q < OB * KS2 ? q : OB * KS2 - 1) * FRAG));
#endif
        mfma3(wh, wl, h1h[ks], h1l[ks], acc, accx);
        // LDS reads in flight bounded (the scheduler would hoist all 16 k-steps' W hi reads)
        if (ks % X3L_GROUP == X3L_GROUP - 1) __builtin_amdgcn_sched_barrier(0);
      }
      acc = x3_sum(acc, accx);
      f16x8 a0h = {}, a1h = {}, a0l = {}, a1l = {};  // lanes n >= out feed logits rows that are never read
      if (w3lane) {  // this block's layer-3 fragments (k-steps 2ob, 2ob+1), the lo halves from L2
        a0h = w3f[(2 * ob) * 2 * out + w3idx];
        a1h = w3f[(2 * ob + 1) * 2 * out + w3idx];
        a0l = wlo_load(WL, 16u * (uint32_t)w3idx, sb + (uint32_t)(L.w3 + (size_t)(2 * ob) * 2 * out * 16));
        a1l = wlo_load(WL, 16u * (uint32_t)w3idx, sb + (uint32_t)(L.w3 + (size_t)(2 * ob + 1) * 2 * out * 16));
      }
      f16x8 h2h, h2l;
      split8(acc, 0, true, h2h, h2l);
      mfma3(a0h, a0l, h2h, h2l, acc3, acc3x);
      split8(acc, 1, true, h2h, h2l);
      mfma3(a1h, a1l, h2h, h2l, acc3, acc3x);
    }
    acc3 = x3_sum(acc3, acc3x);
    // ---- outputs: lane holds logits m = (i&3) + 8(i>>2) + 4h of its row (out <= 12: i < 8)
    if (A.logits && valid) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = (i & 3) + 8 * (i >> 2) + 4 * h;
        if (m < out) A.logits[row * out + m] = acc3[i];
      }
    }
    if (A.actions) {
      float lg[12];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        lg[i] = acc3[i];
        lg[4 + i] = __shfl_xor(acc3[i], 32);
        lg[8 + i] = acc3[4 + i];
      }
      const int ad = out / 2;
      if (h == 0 && valid) {
#pragma unroll
        for (int k = 0; k < 6; ++k)
          if (k < ad) A.actions[row * ad + k] = lg[k];
      }
    }
  }
}

// bf16: 8 waves per workgroup (one workgroup per CU: the LDS blob), one 32-row tile per wave (12 /
// 16 waves and two tiles per wave measured slower)
constexpr int BF16_TILES = 1;
constexpr int BF16_WAVES_T = 8;
constexpr int F32_WAVES = 4;
// f32x3: waves per workgroup (one workgroup per CU: the LDS blob); 4 = one wave per SIMD: the hi
// and lo fragments of h1 (128 registers, lo in AGPRs), the accumulator chains, the double-buffered
// W2 lo batches and the next tile's observations need ~380 registers (at 2 waves per SIMD, 256,
// it spills)
constexpr int X3_WAVES = 4;
// policy_mlp_x3l (two waves per SIMD) unless SWARM_POLICY_X3_PIPELINED=1 is set in the environment
// (the one-wave pipelined kernel; same outputs bit for bit)
constexpr int X3L_WAVES = 8;

thread_local char g_perr[256] = "";
int pfail(int code, const char* msg) {
  strncpy(g_perr, msg, sizeof(g_perr) - 1);
  return code;
}

int grid_for(int waves_per_block, long long tiles) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
      (void)hipGetLastError();
      cus = 256;
    }
  }
  long long need = (tiles + waves_per_block - 1) / waves_per_block;
  long long g = need < cus ? need : cus;
  return g < 1 ? 1 : (int)g;
}

}  // namespace

extern "C" {

const char* swarm_policy_last_error(void) { return g_perr; }

long long swarm_policy_packed_bytes(int in_dim, int out_dim, int precision) {
  if (in_dim < 1 || in_dim > SWARM_POLICY_MAX_IN || out_dim < 2 || out_dim > SWARM_POLICY_MAX_OUT || (out_dim & 1))
    return pfail(SWARM_ELIMIT, "policy dims out of range"), (long long)SWARM_ELIMIT;
  if (precision == SWARM_POLICY_BF16) return (long long)Bf16Layout(out_dim).total;
  if (precision == SWARM_POLICY_F32X3) return 2 * (long long)Bf16Layout(out_dim).total;  // hi blob, lo blob
  if (precision == SWARM_POLICY_F32) return (long long)F32Layout(in_dim).total * 4;
  return pfail(SWARM_EINVAL, "unknown precision"), (long long)SWARM_EINVAL;
}

int swarm_policy_pack(int in_dim, int out_dim, int precision, const float* w1, const float* b1, const float* w2,
                      const float* b2, const float* w3, const float* b3, void* host_out) {
  const long long nb = swarm_policy_packed_bytes(in_dim, out_dim, precision);
  if (nb < 0) return (int)nb;
  if (!w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !host_out) return pfail(SWARM_ENULL, "null weight pointer");
  memset(host_out, 0, (size_t)nb);
  if (precision == SWARM_POLICY_F32X3) {
    // the bf16 blob's fragment order twice, f16 elements: hi = f16(v), then lo = f16((v - hi) 2^11)
    const Bf16Layout L(out_dim);
    for (int part = 0; part < 2; ++part) {
      unsigned char* base = static_cast<unsigned char*>(host_out) + part * L.total;
      auto cv = [part](float v) -> uint16_t {
        const uint16_t hi = f16_rne(v);
        return part == 0 ? hi : f16_rne((v - f16_to_f32(hi)) * 2048.f);  // lo scaled by 2^11 (kernel: X3_LO_SCALE)
      };
      uint16_t* w1f = reinterpret_cast<uint16_t*>(base + L.w1);
      uint16_t* w2f = reinterpret_cast<uint16_t*>(base + L.w2);
      uint16_t* w3f = reinterpret_cast<uint16_t*>(base + L.w3);
      for (int ob = 0; ob < OB; ++ob)
        for (int l = 0; l < 64; ++l) {
          const int m = ob * 32 + (l & 31), h = l >> 5;
          for (int ks = 0; ks < KS1; ++ks)
            for (int j = 0; j < 8; ++j) {
              const int k = 16 * ks + 8 * h + j;
              const float v = k < in_dim ? w1[m * in_dim + k] : (k == in_dim ? b1[m] : 0.f);
              w1f[((ob * KS1 + ks) * 64 + l) * 8 + j] = cv(v);
            }
          for (int ks = 0; ks < KS2; ++ks)
            for (int j = 0; j < 8; ++j) w2f[((ob * KS2 + ks) * 64 + l) * 8 + j] = cv(w2[m * H + chained_k(ks, h, j)]);
        }
      for (int ks = 0; ks < KS2; ++ks)
        for (int h = 0; h < 2; ++h)
          for (int m = 0; m < out_dim; ++m)
            for (int j = 0; j < 8; ++j)
              w3f[((ks * 2 * out_dim) + h * out_dim + m) * 8 + j] = cv(w3[m * H + chained_k(ks, h, j)]);
      if (part == 0) {
        memcpy(base + L.b2, b2, H * 4);
        memcpy(base + L.b3, b3, (size_t)out_dim * 4);
      }
    }
  } else if (precision == SWARM_POLICY_BF16) {
    const Bf16Layout L(out_dim);
    unsigned char* base = static_cast<unsigned char*>(host_out);
    uint16_t* w1f = reinterpret_cast<uint16_t*>(base + L.w1);
    uint16_t* w2f = reinterpret_cast<uint16_t*>(base + L.w2);
    uint16_t* w3f = reinterpret_cast<uint16_t*>(base + L.w3);
    for (int ob = 0; ob < OB; ++ob)
      for (int l = 0; l < 64; ++l) {
        const int m = ob * 32 + (l & 31), h = l >> 5;
        for (int ks = 0; ks < KS1; ++ks)
          for (int j = 0; j < 8; ++j) {
            const int k = 16 * ks + 8 * h + j;
            const float v = k < in_dim ? w1[m * in_dim + k] : (k == in_dim ? b1[m] : 0.f);
            w1f[((ob * KS1 + ks) * 64 + l) * 8 + j] = bf16_rne(v);
          }
        for (int ks = 0; ks < KS2; ++ks)
          for (int j = 0; j < 8; ++j)
            w2f[((ob * KS2 + ks) * 64 + l) * 8 + j] = bf16_rne(w2[m * H + chained_k(ks, h, j)]);
      }
    for (int ks = 0; ks < KS2; ++ks)
      for (int h = 0; h < 2; ++h)
        for (int m = 0; m < out_dim; ++m)
          for (int j = 0; j < 8; ++j)
            w3f[((ks * 2 * out_dim) + h * out_dim + m) * 8 + j] = bf16_rne(w3[m * H + chained_k(ks, h, j)]);
    memcpy(base + L.b2, b2, H * 4);
    memcpy(base + L.b3, b3, (size_t)out_dim * 4);
  } else {
    const F32Layout L(in_dim);
    float* f = static_cast<float*>(host_out);
    for (int ob = 0; ob < 16; ++ob)
      for (int l = 0; l < 64; ++l) {
        const int m = ob * 16 + (l & 15), g = l >> 4;
        for (int q = 0; q < L.kq1; ++q) {
          const int k = 4 * q + g;
          f[L.w1 + ((size_t)ob * L.kq1 + q) * 64 + l] = k < in_dim ? w1[m * in_dim + k] : (k == in_dim ? b1[m] : 0.f);
        }
        for (int q = 0; q < 64; ++q) f[L.w2 + ((size_t)ob * 64 + q) * 64 + l] = w2[m * H + chained_k_f32(q, g)];
      }
    for (int l = 0; l < 64; ++l) {
      const int m = l & 15, g = l >> 4;
      for (int q = 0; q < 64; ++q) f[L.w3 + (size_t)q * 64 + l] = m < out_dim ? w3[m * H + chained_k_f32(q, g)] : 0.f;
    }
    memcpy(f + L.b2, b2, H * 4);
    memcpy(f + L.b3, b3, (size_t)out_dim * 4);
  }
  return SWARM_OK;
}

int swarm_policy_forward(const swarm_policy_t* p, const float* obs, long long rows, float* logits, float* actions,
                         int action_mode, unsigned long long seed, unsigned long long counter, void* hip_stream) {
  if (!p || !p->weights) return pfail(SWARM_ENULL, "policy/weights is NULL");
  if (swarm_policy_packed_bytes(p->in_dim, p->out_dim, p->precision) < 0) return SWARM_ELIMIT;
  if (rows < 0) return pfail(SWARM_EINVAL, "rows < 0");
  if (rows == 0) return SWARM_OK;
  if (!obs) return pfail(SWARM_ENULL, "obs is NULL");
  if (!logits && !actions) return pfail(SWARM_ENULL, "need logits and/or actions");
  if (action_mode != SWARM_POLICY_ACT_MEAN && action_mode != SWARM_POLICY_ACT_SAMPLE)
    return pfail(SWARM_EINVAL, "unknown action_mode");
  if (action_mode == SWARM_POLICY_ACT_SAMPLE && p->precision != SWARM_POLICY_BF16)
    return pfail(SWARM_EINVAL, "sampled actions are implemented on the bf16 path");
  if (((uintptr_t)p->weights) % 16) return pfail(SWARM_EINVAL, "weights must be 16-B aligned");
  FwdArgs a;
  a.w = p->weights;
  a.obs = obs;
  a.logits = logits;
  a.actions = actions;
  a.rows = rows;
  a.in = p->in_dim;
  a.out = p->out_dim;
  a.mode = action_mode;
  a.seed_lo = (uint32_t)seed;
  a.seed_hi = (uint32_t)(seed >> 32);
  a.ctr_lo = (uint32_t)counter;
  a.ctr_hi = (uint32_t)(counter >> 32);
  hipStream_t s = (hipStream_t)hip_stream;
  if (p->precision == SWARM_POLICY_BF16) {
    const int lds = (int)Bf16Layout(p->out_dim).total;
    const bool dflt = p->in_dim == 37 && p->out_dim == 6;  // K = 3, Ms = 4 obs; 3-d Gaussian actions
    auto fn = action_mode == SWARM_POLICY_ACT_SAMPLE
                  ? (dflt ? policy_mlp_bf16<BF16_WAVES_T, SWARM_POLICY_ACT_SAMPLE, BF16_TILES, 37, 6>
                          : policy_mlp_bf16<BF16_WAVES_T, SWARM_POLICY_ACT_SAMPLE, BF16_TILES>)
                  : (dflt ? policy_mlp_bf16<BF16_WAVES_T, SWARM_POLICY_ACT_MEAN, BF16_TILES, 37, 6>
                          : policy_mlp_bf16<BF16_WAVES_T, SWARM_POLICY_ACT_MEAN, BF16_TILES>);
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
        hipSuccess)
      return pfail(SWARM_EHIP, "hipFuncSetAttribute failed");
    const int grid = grid_for(BF16_WAVES_T, ((rows + 31) / 32 + BF16_TILES - 1) / BF16_TILES);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(64 * BF16_WAVES_T), lds, s, a);
  } else if (p->precision == SWARM_POLICY_F32X3) {
    const int lds = (int)Bf16Layout(p->out_dim).total;
    const bool dflt = p->in_dim == 37 && p->out_dim == 6;
    (void)dflt;  // the compile-time-dims instance spills (71 VGPRs at 512); the runtime-dims one fits (492)
    const char* pipe = getenv("SWARM_POLICY_X3_PIPELINED");
    const bool lean = !(pipe && pipe[0] == '1');
    auto fn = lean ? policy_mlp_x3l<X3L_WAVES> : policy_mlp_x3<X3_WAVES>;
    const int waves = lean ? X3L_WAVES : X3_WAVES;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
        hipSuccess)
      return pfail(SWARM_EHIP, "hipFuncSetAttribute failed");
    const int grid = grid_for(waves, (rows + 31) / 32);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(64 * waves), lds, s, a);
  } else {
    const int grid = grid_for(F32_WAVES, (rows + 15) / 16) * 2;
    hipLaunchKernelGGL(policy_mlp_f32<F32_WAVES>, dim3(grid), dim3(64 * F32_WAVES), 0, s, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pfail(SWARM_EHIP, hipGetErrorString(e));
  return SWARM_OK;
}

}  // extern "C"
