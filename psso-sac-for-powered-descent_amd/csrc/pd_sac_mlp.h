// pd_sac_mlp.h -- the SAC actor's forward pass for one tile of 16 envs by one 256-thread
// workgroup (SURVEY 8f rank 3's caller).  Used by pd_sac_actor (pdsac.hip, its own launch) and by
// the c5 step kernel's prologue (k_step<..., SAC>, pd_step_sac_fused: one launch per step).
//
// Actor.forward (sac_pytorch.py:129-159): shared_net = Linear(S, H) ReLU [Linear(H, H) ReLU] x
// (n_hidden_layers - 1), then the mean and log_std heads Linear(H, A) (the clamp of log_std and
// the sampling are the step kernel's).  Activations stay in LDS:
//   layer 1 (K = S <= 16): VALU fmaf chains, one output per thread per pass;
//   hidden layers (H x H):  v_mfma_f32_16x16x4_f32 (exact f32 products, one rounding per
//                           k-ordered fma step), the 16 envs as rows, 16 output columns per tile,
//                           two tiles in flight per wave; the weight rows stream from L2 as float4
//                           per lane, the activations come from LDS as float4 per lane;
//   heads (A outputs each): 16 lanes per env split the H-term dots, a shuffle tree adds them.
// Numerics: f32 throughout (the reference's dtype); the sums run in another order than
// hipBLASLt's (both are f32 GEMMs of the same Linear layers), so the heads agree with torch's to
// f32 rounding, not bit for bit (tests/test_gpu_parity.py bounds it).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace pd {

constexpr int kSacBlock = 256;     // 4 waves
constexpr int kSacTile = 16;       // envs per tile (the MFMA's 16 rows)
constexpr int kSacMaxLayers = 8;

struct SacMlp {
    int S, L, A, H;
    const float* obs;                    // [n][S]
    const float* w[kSacMaxLayers];       // w[0] [H][S], w[l] [H][H]
    const float* b[kSacMaxLayers];       // [H]
    const float* wm; const float* bm;    // mean head [A][H], [A]
    const float* ws; const float* bs;    // log_std head
};

using f32x4 = __attribute__((ext_vector_type(4))) float;

// LDS floats the tile needs: two activation buffers of 16 rows, row pitch H + 4 (rows start 4
// banks apart)
template <int H> constexpr int sac_mlp_lds_floats() { return 2 * kSacTile * (H + 4); }

// Envs e0 .. e0 + 15 (rows past n read a zero observation); put(e, o, v): head output o
// (0 .. A-1 mean, A .. 2A-1 log_std, unclamped) of tile row e.  Called by all 256 threads of
// the workgroup (it synchronises them); hb: sac_mlp_lds_floats<H>() floats of LDS.  MA: SacMlp
// in any address space (the step kernel reads it from its kernarg segment).  mark(k): called by
// every thread at the end of phase k (0 layer 1, l hidden layer l, L the heads) -- the section
// clocks of tools/mlp_clocks.hip; the product passes none.
struct NoMark { __device__ void operator()(int) const {} };
template <int H, typename MA, typename Put, typename Mark = NoMark>
__device__ __forceinline__ void sac_mlp_tile(const MA& a, int64_t n, int64_t e0, float* hb, Put&& put,
                                             Mark&& mark = Mark{}) {
    constexpr int P = H + 4;
    float* h0 = hb;
    float* h1 = hb + kSacTile * P;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // ---- layer 1: h[e][j] = relu(sum_k obs[e][k] W1[j][k] + b1[j])
    for (int idx = tid; idx < kSacTile * H; idx += kSacBlock) {
        const int e = idx / H, j = idx - e * H;
        const int64_t ge = e0 + e;
        float acc = 0.f;
        for (int k = 0; k < a.S; ++k) acc = fmaf(ge < n ? a.obs[ge * a.S + k] : 0.f, a.w[0][j * a.S + k], acc);
        acc += a.b[0][j];
        h0[e * P + j] = acc < 0.f ? 0.f : acc;
    }
    __syncthreads();
    mark(0);
    // ---- hidden layers on MFMA: wave w computes the column tiles w, w + 4, ... two at a time
    const int r = lane & 15, q = lane >> 4;
    float* hin = h0;
    float* hout = h1;
    for (int l = 1; l < a.L; ++l) {
        const float* W = a.w[l];
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
        mark(l);
        float* tmp = hin; hin = hout; hout = tmp;
    }
    // ---- heads: env e = tid / 16, part p = tid % 16 sums k in [p H/16, (p + 1) H/16) of each of
    // the 2A outputs; a shuffle tree over the 16 parts
    const float* h = hin;
    const int e = tid >> 4, p = tid & 15;
    for (int o = 0; o < 2 * a.A; ++o) {
        const float* wr = o < a.A ? a.wm + (size_t)o * H : a.ws + (size_t)(o - a.A) * H;
        float acc = 0.f;
#pragma unroll 4
        for (int k = p * (H / 16); k < (p + 1) * (H / 16); ++k) acc = fmaf(h[e * P + k], wr[k], acc);
        acc += __shfl_xor(acc, 8, 16);
        acc += __shfl_xor(acc, 4, 16);
        acc += __shfl_xor(acc, 2, 16);
        acc += __shfl_xor(acc, 1, 16);
        if (p == 0) put(e, o, acc + (o < a.A ? a.bm[o] : a.bs[o - a.A]));
    }
    mark(a.L);
}

}  // namespace pd
