// pdsac.hip -- the SAC actor of the c5 collection step as one kernel (SURVEY 8f rank 3's caller).
//
// Actor.forward (sac_pytorch.py:129-159): shared_net = Linear(S, H) ReLU [Linear(H, H) ReLU] x
// (n_hidden_layers - 1), then the mean and log_std heads Linear(H, A) (the clamp of log_std and
// the sampling are pd_step_sac's).  PyTorch runs it as 2 + L GEMM launches (hipBLASLt) plus the
// ReLUs; here one launch computes the whole MLP for a tile of 16 envs per workgroup, keeping the
// activations in LDS:
//   layer 1 (K = S <= 16): VALU fmaf chains, one output per thread per pass;
//   hidden layers (H x H):  v_mfma_f32_16x16x4_f32 (exact f32 products, one rounding per
//                           k-ordered fma step), the 16 envs as rows, 16 output columns per tile,
//                           two tiles in flight per wave; the weight rows stream from L2 as float4
//                           per lane, the activations come from LDS as float4 per lane;
//   heads (A outputs each): 16 lanes per env split the H-term dots, a shuffle tree adds them.
// Numerics: f32 throughout (the reference's dtype); the sums run in another order than
// hipBLASLt's (both are f32 GEMMs of the same Linear layers), so the heads agree with torch's to
// f32 rounding, not bit for bit (tests/test_gpu_drivers.py bounds it).
#include <hip/hip_runtime.h>

#include "../../include/pdenv.h"

namespace {

constexpr int kActorBlock = 256;   // 4 waves
constexpr int kEnvTile = 16;       // envs per workgroup (the MFMA's 16 rows)
constexpr int kMaxLayers = 8;

struct ActorArgs {
    int64_t n;
    int S, L, A;
    const float* obs;            // [n][S]
    const float* w[kMaxLayers];  // w[0] [H][S], w[l] [H][H]
    const float* b[kMaxLayers];  // [H]
    const float* wm; const float* bm;   // mean head [A][H], [A]
    const float* ws; const float* bs;   // log_std head
    float* heads;                // [n][2A]: mean | log_std (unclamped)
};

using f32x4 = __attribute__((ext_vector_type(4))) float;

template <int H>
__global__ __launch_bounds__(kActorBlock) void k_sac_actor(ActorArgs a) {
    constexpr int P = H + 4;   // LDS row pitch (floats): rows start 4 banks apart
    __shared__ __attribute__((aligned(16))) float hb[2][kEnvTile * P];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t e0 = (int64_t)blockIdx.x * kEnvTile;
    // ---- layer 1: h[e][j] = relu(sum_k obs[e][k] W1[j][k] + b1[j])
    for (int idx = tid; idx < kEnvTile * H; idx += kActorBlock) {
        const int e = idx / H, j = idx - e * H;
        const int64_t ge = e0 + e;
        float acc = 0.f;
        for (int k = 0; k < a.S; ++k) acc = fmaf(ge < a.n ? a.obs[ge * a.S + k] : 0.f, a.w[0][j * a.S + k], acc);
        acc += a.b[0][j];
        hb[0][e * P + j] = acc < 0.f ? 0.f : acc;
    }
    __syncthreads();
    // ---- hidden layers on MFMA: wave w computes the column tiles w, w + 4, ... two at a time
    const int r = lane & 15, q = lane >> 4;
    int cur = 0;
    for (int l = 1; l < a.L; ++l) {
        const float* W = a.w[l];
        const float* hin = hb[cur];
        float* hout = hb[cur ^ 1];
        for (int t = wave; t < H / 16; t += 8) {
            const int t2 = t + 4;   // (H / 16 is a multiple of 8: both tiles exist)
            f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
            const float* w0 = W + (size_t)(16 * t + r) * H + 4 * q;
            const float* w1 = W + (size_t)(16 * t2 + r) * H + 4 * q;
            // k in chunks of KC x 16: the tile pair's weight fragments of a chunk first (global
            // loads in flight together, 2 KC float4 registers), then its 8 KC MFMAs
            constexpr int KC = H / 16 < 16 ? H / 16 : 16;
#pragma unroll 1
            for (int k0 = 0; k0 < H / 16; k0 += KC) {
                f32x4 b0[KC], b1[KC];
#pragma unroll
                for (int kb = 0; kb < KC; ++kb) {
                    b0[kb] = *(const f32x4*)(w0 + 16 * (k0 + kb));
                    b1[kb] = *(const f32x4*)(w1 + 16 * (k0 + kb));
                }
                // (keep the loads together ahead of the MFMAs: the scheduler would otherwise
                // sink each next to its first use, leaving two or three in flight)
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int kb = 0; kb < KC; ++kb) {
                    const f32x4 av = *(const f32x4*)(hin + r * P + 16 * (k0 + kb) + 4 * q);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], b0[kb][j], c0, 0, 0, 0);
                        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], b1[kb][j], c1, 0, 0, 0);
                    }
                }
            }
            // D[row 4q + i][col r] + bias, relu, into the next activation tile
            const float bb0 = a.b[l][16 * t + r], bb1 = a.b[l][16 * t2 + r];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float v0 = c0[i] + bb0, v1 = c1[i] + bb1;
                hout[(4 * q + i) * P + 16 * t + r] = v0 < 0.f ? 0.f : v0;
                hout[(4 * q + i) * P + 16 * t2 + r] = v1 < 0.f ? 0.f : v1;
            }
        }
        __syncthreads();
        cur ^= 1;
    }
    // ---- heads: env e = tid / 16, part p = tid % 16 sums k in [p H/16, (p + 1) H/16) of each of
    // the 2A outputs; a shuffle tree over the 16 parts
    const float* h = hb[cur];
    const int e = tid >> 4, p = tid & 15;
    const int64_t ge = e0 + e;
    for (int o = 0; o < 2 * a.A; ++o) {
        const float* wr = o < a.A ? a.wm + (size_t)o * H : a.ws + (size_t)(o - a.A) * H;
        float acc = 0.f;
#pragma unroll 4
        for (int k = p * (H / 16); k < (p + 1) * (H / 16); ++k) acc = fmaf(h[e * P + k], wr[k], acc);
        acc += __shfl_xor(acc, 8, 16);
        acc += __shfl_xor(acc, 4, 16);
        acc += __shfl_xor(acc, 2, 16);
        acc += __shfl_xor(acc, 1, 16);
        if (p == 0 && ge < a.n) a.heads[ge * 2 * a.A + o] = acc + (o < a.A ? a.bm[o] : a.bs[o - a.A]);
    }
}

}  // namespace

namespace pd {
pd_status set_error(pd_status s, const char* m);   // pdenv.hip: the pd_last_error() message
}

extern "C" {

pd_status pd_sac_actor(int64_t n, int32_t state_dim, int32_t hidden, int32_t n_hidden_layers, int32_t action_dim,
                       const float* obs, const float* const* params, float* heads, void* stream) {
    if (n < 0 || state_dim < 1 || state_dim > 16 || n_hidden_layers < 1 || n_hidden_layers > kMaxLayers ||
        action_dim < 1 || action_dim > 8 || !params || !heads || (n > 0 && !obs))
        return pd::set_error(PD_ERR_INVALID, "pd_sac_actor: bad arguments");
    if (hidden != 128 && hidden != 256 && hidden != 512)
        return pd::set_error(PD_ERR_UNSUPPORTED, "pd_sac_actor: hidden width 128, 256 or 512 only");
    if (n == 0) return PD_OK;
    ActorArgs a{};
    a.n = n; a.S = state_dim; a.L = n_hidden_layers; a.A = action_dim; a.obs = obs; a.heads = heads;
    for (int l = 0; l < n_hidden_layers; ++l) {
        a.w[l] = params[2 * l]; a.b[l] = params[2 * l + 1];
        if (!a.w[l] || !a.b[l]) return pd::set_error(PD_ERR_INVALID, "pd_sac_actor: null layer parameter");
    }
    a.wm = params[2 * n_hidden_layers]; a.bm = params[2 * n_hidden_layers + 1];
    a.ws = params[2 * n_hidden_layers + 2]; a.bs = params[2 * n_hidden_layers + 3];
    if (!a.wm || !a.bm || !a.ws || !a.bs) return pd::set_error(PD_ERR_INVALID, "pd_sac_actor: null head parameter");
    const dim3 grid((unsigned)((n + kEnvTile - 1) / kEnvTile));
    hipStream_t s = (hipStream_t)stream;
    switch (hidden) {
        case 128: hipLaunchKernelGGL(k_sac_actor<128>, grid, dim3(kActorBlock), 0, s, a); break;
        case 512: hipLaunchKernelGGL(k_sac_actor<512>, grid, dim3(kActorBlock), 0, s, a); break;
        default: hipLaunchKernelGGL(k_sac_actor<256>, grid, dim3(kActorBlock), 0, s, a); break;
    }
    if (hipGetLastError() != hipSuccess) return pd::set_error(PD_ERR_HIP, "pd_sac_actor: launch failed");
    return PD_OK;
}

}  // extern "C"
