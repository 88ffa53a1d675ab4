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
// in any address space (the step kernel reads it from its kernarg segment).
//
// Latency plan (one wave per SIMD in the c5 step kernel, so nothing else hides a round trip):
//   - every global load of a phase is issued before its first use: the heads' weights first (held
//     in registers through the hidden layers, stored into the free activation buffer after them),
//     layer 1's column weights and the tile's observations together;
//   - a hidden layer's wave keeps all its column tiles in flight (2 / 4 / 8 for H = 128 / 256 /
//     512, at most 4 at a time) and streams their weight fragments kD k-blocks ahead of the MFMAs,
//     so the MFMA pipe (32 cycles per v_mfma_f32_16x16x4_f32, 40 of dependent latency) is the
//     bound, not the L2;
// with every sum in the order of the straightforward loops (layer 1: k ascending then the bias;
// the MFMA k-blocks ascending; the heads' 16 partial sums by a shuffle tree), so pd_sac_actor and
// the fused step kernel, which share this function, give the same bits.
template <int H, typename MA, typename Put>
__device__ __forceinline__ void sac_mlp_tile(const MA& a, int64_t n, int64_t e0, float* hb, Put&& put) {
    constexpr int P = H + 4;
    float* h0 = hb;
    float* h1 = hb + kSacTile * P;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int S = a.S, A = a.A;
    // ---- the heads' weights (mean rows then log_std rows, [2A][H]): requested now, kept in
    // registers through the hidden layers (at most 2 8 H / 256 floats per thread)
    constexpr int kHW = 2 * 8 * H / kSacBlock;
    float hw[kHW];
    const int nhw = 2 * A * H;
#pragma unroll
    for (int i = 0; i < kHW; ++i) {
        const int idx = tid + i * kSacBlock;
        hw[i] = idx < A * H ? a.wm[idx] : (idx < nhw ? a.ws[idx - A * H] : 0.f);
    }
    // ---- layer 1: h[e][j] = relu(sum_k obs[e][k] W1[j][k] + b1[j]): the tile's observations into
    // LDS (h1 is free until the first hidden layer), each thread's columns' weights in registers
    constexpr int kCols1 = (H + kSacBlock - 1) / kSacBlock;
    float w1[kCols1][16], b1[kCols1];
#pragma unroll
    for (int c = 0; c < kCols1; ++c) {
        const int j = tid + c * kSacBlock;
#pragma unroll
        for (int k = 0; k < 16; ++k) w1[c][k] = (j < H && k < S) ? a.w[0][j * S + k] : 0.f;
        b1[c] = j < H ? a.b[0][j] : 0.f;
    }
    if (tid < kSacTile * S) {
        const int e = tid / S;
        h1[tid] = e0 + e < n ? a.obs[(e0 + e) * S + (tid - e * S)] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kCols1; ++c) {
        const int j = tid + c * kSacBlock;
        if (j < H) {
#pragma unroll 4
            for (int e = 0; e < kSacTile; ++e) {
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < 16; ++k) if (k < S) acc = fmaf(h1[e * S + k], w1[c][k], acc);
                acc += b1[c];
                h0[e * P + j] = acc < 0.f ? 0.f : acc;
            }
        }
    }
    __syncthreads();
    // ---- hidden layers on MFMA: wave w computes the column tiles w, w + 4, ..., NT at a time,
    // their weight fragments kD k-blocks (of 16) ahead of the MFMAs that use them
    const int r = lane & 15, q = lane >> 4;
    float* hin = h0;
    float* hout = h1;
    constexpr int kTiles = H / 16 / 4;                 // column tiles per wave
    constexpr int NT = kTiles < 4 ? kTiles : 4;        // in flight together
    constexpr int KB = H / 16;                         // k-blocks
    constexpr int kD = 4;                              // prefetch distance (k-blocks)
    for (int l = 1; l < a.L; ++l) {
        const float* W = a.w[l];
#pragma unroll 1
        for (int g = 0; g < kTiles; g += NT) {
            f32x4 c[NT];
            const float* wp[NT];
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                c[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                wp[i] = W + (size_t)(16 * (wave + 4 * (g + i)) + r) * H + 4 * q;
            }
            f32x4 bw[kD][NT];
#pragma unroll
            for (int kb = 0; kb < kD && kb < KB; ++kb)
#pragma unroll
                for (int i = 0; i < NT; ++i) bw[kb][i] = *(const f32x4*)(wp[i] + 16 * kb);
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                const f32x4 av = *(const f32x4*)(hin + r * P + 16 * kb + 4 * q);
                f32x4 cur[NT];
#pragma unroll
                for (int i = 0; i < NT; ++i) cur[i] = bw[kb % kD][i];
                if (kb + kD < KB) {
#pragma unroll
                    for (int i = 0; i < NT; ++i) bw[kb % kD][i] = *(const f32x4*)(wp[i] + 16 * (kb + kD));
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int i = 0; i < NT; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], cur[i][j], c[i], 0, 0, 0);
                // (the next block's loads stay behind this block's MFMAs, kD blocks ahead: the
                // scheduler would otherwise hoist every load of the unrolled loop to the top)
                __builtin_amdgcn_sched_barrier(0);
            }
            // D[row 4q + i][col r] + bias, relu, into the next activation tile
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                const int col = 16 * (wave + 4 * (g + i)) + r;
                const float bb = a.b[l][col];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const float v = c[i][m] + bb;
                    hout[(4 * q + m) * P + col] = v < 0.f ? 0.f : v;
                }
            }
        }
        __syncthreads();
        float* tmp = hin; hin = hout; hout = tmp;
    }
    // ---- heads: their weights into the free activation buffer, then env e = tid / 16, part
    // p = tid % 16 sums k in [p H/16, (p + 1) H/16) of each of the 2A outputs; a shuffle tree over
    // the 16 parts
    float* hwl = hout;
#pragma unroll
    for (int i = 0; i < kHW; ++i) {
        const int idx = tid + i * kSacBlock;
        if (idx < nhw) hwl[idx] = hw[i];
    }
    __syncthreads();
    const float* h = hin;
    const int e = tid >> 4, p = tid & 15;
    for (int o = 0; o < 2 * A; ++o) {
        const float* wr = hwl + o * H;
        float acc = 0.f;
#pragma unroll
        for (int k = p * (H / 16); k < (p + 1) * (H / 16); ++k) acc = fmaf(h[e * P + k], wr[k], acc);
        acc += __shfl_xor(acc, 8, 16);
        acc += __shfl_xor(acc, 4, 16);
        acc += __shfl_xor(acc, 2, 16);
        acc += __shfl_xor(acc, 1, 16);
        if (p == 0) put(e, o, acc + (o < A ? a.bm[o] : a.bs[o - A]));
    }
}

}  // namespace pd
