// mlp.hip — fused MLP gradient step for the iterative DP-SGD workload
// (the APRIL-ANN example of the reference: "256 inputs 128 tanh 10 log_softmax",
// multi-class cross-entropy, bunch 128 —
// /root/reference/mapreduce/examples/APRIL-ANN/init.lua:10-12,127-141 and the
// map/reduce/final functions in examples/APRIL-ANN/common.lua:85-202).
//
// One launch computes, for a bunch of B gathered patterns, the forward pass,
// the loss, and the gradient of the SUMMED loss w.r.t. every parameter:
//
//   H  = tanh(X W1 + b1)            X:[B,IN]  W1:[IN,HID]     (MFMA f32 16x16x4)
//   Z  = H W2 + b2                  W2:[HID,OUT]              (VALU, OUT = 10)
//   L  = sum_r  logsumexp(Z_r) - Z_r[y_r]
//   dZ = softmax(Z) - onehot(y)
//   dW2 = H^T dZ, db2 = sum dZ, dH = (dZ W2^T) * (1 - H^2)
//   dW1 = X^T dH                    K = 16 rows per block     (MFMA f32 16x16x4)
//   db1 = sum dH
//
// Each block owns 16 rows of the bunch (4 waves; wave w owns hidden columns
// [32w, 32w+32)).  X rows are gathered straight from the HBM-resident dataset by
// index (no host-side batch assembly) into LDS, H and dH stay in LDS, and the
// per-block parameter gradients go to a workspace; a second, chip-wide kernel
// folds them in fixed block order (deterministic, no atomics).  Both launches
// are capture-safe (no host synchronisation).
//
// f32-in MFMA on gfx950 is exact f32 (a k-ordered fmaf chain), so results match
// a PyTorch fp32 reference to rounding.  The optimizer step (SGD + momentum +
// weight decay + the reference's 1/sqrt(N) gradient smoothing, common.lua:161-165)
// is a second, element-wise kernel over the flat parameter vector.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int MLP_ROWS = 16;      // bunch rows per block (MFMA M for the forward GEMM)
constexpr int MLP_THREADS = 256;  // 4 waves

template <int IN, int HID, int OUT>
struct MlpLayout {
  static constexpr int W1 = 0;
  static constexpr int B1 = IN * HID;
  static constexpr int W2 = B1 + HID;
  static constexpr int B2 = W2 + HID * OUT;
  static constexpr int P = B2 + OUT;
};

template <int IN, int HID, int OUT>
__global__ __launch_bounds__(MLP_THREADS) void mlp_grad_kernel(
    const float* __restrict__ X, const int* __restrict__ labels, const int* __restrict__ idx, int B,
    const float* __restrict__ params, float* __restrict__ grads, float* __restrict__ loss_out,
    float* __restrict__ partials, unsigned* __restrict__ counter, int do_grad) {
  using Lay = MlpLayout<IN, HID, OUT>;
  static_assert(HID == 128 && IN % 16 == 0 && OUT <= 16, "layout assumes 4 waves x 32 hidden columns");
  constexpr int XS = IN + 4;   // padded LDS row strides (bank spread)
  constexpr int HS = HID + 4;
  __shared__ float Xs[MLP_ROWS][XS];
  __shared__ float Hs[MLP_ROWS][HS];
  __shared__ float dHs[MLP_ROWS][HS];
  __shared__ float Zs[MLP_ROWS][OUT];
  __shared__ float dZs[MLP_ROWS][OUT];
  __shared__ float rowloss[MLP_ROWS];
  __shared__ float rowok[MLP_ROWS];
  __shared__ int ys[MLP_ROWS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r0 = blockIdx.x * MLP_ROWS;
  const int nrows = min(MLP_ROWS, B - r0);

  // gather the block's 16 rows (float4 per thread-step) into LDS
  for (int e = tid; e < MLP_ROWS * (IN / 4); e += MLP_THREADS) {
    const int r = e / (IN / 4), c4 = e % (IN / 4);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (r < nrows) v = *reinterpret_cast<const f32x4*>(X + (size_t)idx[r0 + r] * IN + 4 * c4);
    Xs[r][4 * c4 + 0] = v.x;
    Xs[r][4 * c4 + 1] = v.y;
    Xs[r][4 * c4 + 2] = v.z;
    Xs[r][4 * c4 + 3] = v.w;
  }
  if (tid < MLP_ROWS) ys[tid] = tid < nrows ? labels[idx[r0 + tid]] : 0;
  __syncthreads();

  // ---- H = tanh(X W1 + b1): wave owns columns [32w, 32w+32) as two 16x16 tiles
  {
    const float* W1 = params + Lay::W1;
    const int kr = lane >> 4, c = lane & 15;
    const int col0 = wave * 32 + c, col1 = col0 + 16;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int k0 = 0; k0 < IN; k0 += 4) {
      const float a = Xs[c][k0 + kr];
      const float b0 = W1[(size_t)(k0 + kr) * HID + col0];
      const float b1 = W1[(size_t)(k0 + kr) * HID + col1];
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b1, acc1, 0, 0, 0);
    }
    const float bb0 = params[Lay::B1 + col0], bb1 = params[Lay::B1 + col1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = kr * 4 + i;  // C/D map: col = lane&15, row = (lane>>4)*4 + reg
      Hs[row][col0] = tanhf(acc0[i] + bb0);
      Hs[row][col1] = tanhf(acc1[i] + bb1);
    }
  }
  __syncthreads();

  // ---- Z = H W2 + b2 (16 x OUT outputs, K = HID; VALU)
  for (int e = tid; e < MLP_ROWS * OUT; e += MLP_THREADS) {
    const int r = e / OUT, o = e % OUT;
    float z = params[Lay::B2 + o];
    const float* W2 = params + Lay::W2;
#pragma unroll 8
    for (int j = 0; j < HID; ++j) z = fmaf(Hs[r][j], W2[j * OUT + o], z);
    Zs[r][o] = z;
  }
  __syncthreads();

  // ---- log-softmax loss, accuracy and dZ, one thread per row
  if (tid < MLP_ROWS) {
    const int r = tid;
    float m = Zs[r][0];
    int am = 0;
    for (int o = 1; o < OUT; ++o)
      if (Zs[r][o] > m) { m = Zs[r][o]; am = o; }
    float s = 0.f;
    for (int o = 0; o < OUT; ++o) s += expf(Zs[r][o] - m);
    const float lse = m + logf(s);
    const bool live = r < nrows;
    const int y = ys[r];
    rowloss[r] = live ? lse - Zs[r][y] : 0.f;
    rowok[r] = (live && am == y) ? 1.f : 0.f;
    for (int o = 0; o < OUT; ++o) dZs[r][o] = live ? expf(Zs[r][o] - lse) - (o == y ? 1.f : 0.f) : 0.f;
  }
  __syncthreads();

  float* part = partials + (size_t)blockIdx.x * (Lay::P + 2);
  if (tid == 0) {
    float l = 0.f, ok = 0.f;
    for (int r = 0; r < MLP_ROWS; ++r) { l += rowloss[r]; ok += rowok[r]; }
    part[Lay::P] = l;
    part[Lay::P + 1] = ok;
  }

  if (do_grad) {
    // ---- dW2 = H^T dZ, db2 = sum dZ (K = 16)
    for (int e = tid; e < HID * OUT; e += MLP_THREADS) {
      const int j = e / OUT, o = e % OUT;
      float g = 0.f;
#pragma unroll
      for (int r = 0; r < MLP_ROWS; ++r) g = fmaf(Hs[r][j], dZs[r][o], g);
      part[Lay::W2 + e] = g;
    }
    if (tid < OUT) {
      float g = 0.f;
      for (int r = 0; r < MLP_ROWS; ++r) g += dZs[r][tid];
      part[Lay::B2 + tid] = g;
    }
    // ---- dH = (dZ W2^T) * (1 - H^2)
    for (int e = tid; e < MLP_ROWS * HID; e += MLP_THREADS) {
      const int r = e / HID, j = e % HID;
      const float* W2 = params + Lay::W2 + j * OUT;
      float g = 0.f;
#pragma unroll
      for (int o = 0; o < OUT; ++o) g = fmaf(dZs[r][o], W2[o], g);
      const float h = Hs[r][j];
      dHs[r][j] = g * (1.f - h * h);
    }
    __syncthreads();
    if (tid < HID) {
      float g = 0.f;
      for (int r = 0; r < MLP_ROWS; ++r) g += dHs[r][tid];
      part[Lay::B1 + tid] = g;
    }
    // ---- dW1 = X^T dH: (IN/16) x (HID/16) tiles of 16x16, K = 16 rows, MFMA
    {
      const int kr = lane >> 4, c = lane & 15;
      constexpr int MT = IN / 16, NT = HID / 16;
      for (int t = wave; t < MT * NT; t += MLP_THREADS / 64) {
        const int mt = t / NT, nt = t % NT;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k0 = 0; k0 < MLP_ROWS; k0 += 4) {
          const float a = Xs[k0 + kr][mt * 16 + c];   // A = X^T: A[m][k] = X[k][m]
          const float b = dHs[k0 + kr][nt * 16 + c];  // B = dH:  B[k][n]
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = mt * 16 + kr * 4 + i, n = nt * 16 + c;
          part[Lay::W1 + (size_t)m * HID + n] = acc[i];
        }
      }
    }
  }

}

// Fold the per-block partials in block order (deterministic): one thread per
// parameter (+2 loss slots), so the fold is spread over the whole chip (a
// last-block fold by ONE workgroup cost 0.3 ms at B=128 and grew with B).
__global__ void __launch_bounds__(256) mlp_fold_kernel(const float* __restrict__ partials, int nb, int P,
                                                       float* __restrict__ grads, float* __restrict__ loss_out,
                                                       int do_grad) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P + 2 || (!do_grad && p < P)) return;
  float g = 0.f;
  for (int b = 0; b < nb; ++b) g += partials[(size_t)b * (P + 2) + p];
  if (p < P) grads[p] = g;
  else loss_out[p - P] = g;
}

// w <- w + v,  v <- momentum * v - lr * (scale * g + wd * decay(p) * w)
// decay(p) = 1 on weight matrices, 0 on biases (common.lua / init.lua:47:
// "it is better to avoid BIAS regularization").
__global__ void mlp_sgd_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ v, int P,
                               float lr, float momentum, float wd, float scale, int b1_lo, int b1_hi, int b2_lo) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const bool is_bias = (p >= b1_lo && p < b1_hi) || p >= b2_lo;
  const float wp = w[p];
  const float d = scale * g[p] + (is_bias ? 0.f : wd * wp);
  const float vn = momentum * v[p] - lr * d;
  v[p] = vn;
  w[p] = wp + vn;
}

}  // namespace

extern "C" {

int mr_mlp_param_count(int in, int hid, int out) { return in * hid + hid + hid * out + out; }
int mr_mlp_rows_per_block() { return MLP_ROWS; }

// partials: ceil(B/16) * (P + 2) floats; counter: unused (kept for ABI stability).
int mr_mlp_grad(const void* X, const void* labels, const void* idx, int B, int in, int hid, int out,
                const void* params, void* grads, void* loss_out, void* partials, void* counter, int do_grad,
                hipStream_t s) {
  if (in != 256 || hid != 128 || out != 10) return -2;  // the reference's "256 inputs 128 tanh 10 log_softmax"
  if (B <= 0) return 0;
  const int nb = (B + MLP_ROWS - 1) / MLP_ROWS;
  hipLaunchKernelGGL((mlp_grad_kernel<256, 128, 10>), dim3(nb), dim3(MLP_THREADS), 0, s, (const float*)X,
                     (const int*)labels, (const int*)idx, B, (const float*)params, (float*)grads, (float*)loss_out,
                     (float*)partials, (unsigned*)counter, do_grad);
  const int P = MlpLayout<256, 128, 10>::P;
  hipLaunchKernelGGL(mlp_fold_kernel, dim3((P + 2 + 255) / 256), dim3(256), 0, s, (const float*)partials, nb, P,
                     (float*)grads, (float*)loss_out, do_grad);
  return (int)hipGetLastError();
}

int mr_mlp_sgd(void* w, const void* g, void* v, int P, float lr, float momentum, float wd, float scale, int b1_lo,
               int b1_hi, int b2_lo, hipStream_t s) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(mlp_sgd_kernel, dim3((P + 255) / 256), dim3(256), 0, s, (float*)w, (const float*)g, (float*)v, P,
                     lr, momentum, wd, scale, b1_lo, b1_hi, b2_lo);
  return (int)hipGetLastError();
}

}  // extern "C"
