// pd_sac_mlp.h -- the SAC actor's forward pass for one tile of 16 envs by one 256-thread
// workgroup (SURVEY 8f rank 3's caller).  Used by pd_sac_actor (pdsac.hip, its own launch) and by
// the c5 step kernel's prologue (k_step<..., SAC>, pd_step_sac_fused: one launch per step).
//
// Actor.forward (sac_pytorch.py:129-159): shared_net = Linear(S, H) ReLU [Linear(H, H) ReLU] x
// (n_hidden_layers - 1), then the mean and log_std heads Linear(H, A) (the clamp of log_std and
// the sampling are the step kernel's).  Activations stay in LDS:
//   layer 1 (K = S <= 16): each thread owns output columns (their S weights and bias in
//                           registers) and runs the 16 envs of the tile, whose observations are
//                           staged in LDS: one round of global loads, not one per output;
//   hidden layers (H x H):  v_mfma_f32_16x16x4_f32 (exact f32 products, one rounding per
//                           k-ordered fma step), the 16 envs as rows, 16 output columns per tile,
//                           two column tiles of a wave in flight; k runs in blocks of 32, lane
//                           group q taking k = 32 b + 8 q + j (j = 0..7).  The weights reach the
//                           MFMAs through a wave-private LDS ring filled by LDS DMA: each wave
//                           instruction moves 1 KB of whole 128-byte row segments, the next block
//                           in flight during this block's MFMAs, and the fragments are read back
//                           (XOR-swizzled, conflict-free).  Loaded straight into the MFMA layout
//                           (16 rows x 64 bytes per wave instruction) the weights took 17.4 k
//                           cycles a layer on their own, against 6.9 k for the same bytes read
//                           contiguously (tools/mlp_clocks.hip);
//   heads (A outputs each): 16 lanes per env split the H-term dots (their weights and biases
//                           requested at the start and held in registers when they fit), a
//                           shuffle tree adds them.
// Occupancy and waits: in the fused c5 step kernel (LPE 16, binary32 state I/O) the ring takes
// the workgroup's LDS to ~100 KB, so a CU holds one such workgroup: one wave per SIMD
// (profiles/r05_resource_usage.txt, the SAC LPE-16 rows).  Each k-block waits for its ring
// fill with s_waitcnt vmcnt(0), which also drains the env-state and table-staging loads the
// step kernel issued ahead of the actor; the c5 gain of the ring was measured with both costs
// in it.  A partial count cannot keep those loads in flight: vmcnt
// counts vector-memory loads, the LDS DMA fills among them, retiring in issue order, so a wait
// for a ring fill is a wait for every load issued before it.
// Numerics: f32 throughout (the reference's dtype); the sums run in another order than
// hipBLASLt's (both are f32 GEMMs of the same Linear layers), so the heads agree with torch's to
// f32 rounding, not bit for bit (tests/test_gpu_parity.py bounds it).  pd_sac_actor and the fused
// step kernel share this function and give the same bits.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

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
// banks apart), and per wave two 4 KB blocks of weight rows (the hidden layers' LDS DMA ring)
template <int H> constexpr int sac_mlp_lds_floats() {
    return 2 * kSacTile * (H + 4) + 4 * 2 * (H / 64 < 2 ? H / 64 : 2) * 16 * 32;   // + the waves' weight rings
}

// Envs e0 .. e0 + 15 (rows past n read a zero observation); put(e, o, v): head output o
// (0 .. A-1 mean, A .. 2A-1 log_std, unclamped) of tile row e.  Called by all 256 threads of
// the workgroup (it synchronises them); hb: sac_mlp_lds_floats<H>() floats of LDS (a __shared__
// array: the LDS DMA of the hidden layers addresses it as LDS).  MA: SacMlp
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
    const int S = a.S, A = a.A;
    // ---- the heads' weights of this thread's part (env e = tid / 16, part p = tid % 16: k in
    // [p H/16, (p + 1) H/16) of each of the 2A outputs), requested first and held through the
    // hidden layers when the 2A outputs' KP floats fit kHeadRegs (c5: 2 x 16); else read where used
    constexpr int KP = H / 16;
    constexpr int kHeadRegs = 32;
    constexpr int kMaxO = kHeadRegs / KP > 0 ? kHeadRegs / KP : 1;
    const bool heads_early = 2 * A <= kHeadRegs / KP;
    const int e = tid >> 4, p = tid & 15;
    f32x4 hw[kHeadRegs / 4];
    float hb_bias[kMaxO];
#pragma unroll
    for (int o = 0; o < kMaxO; ++o) hb_bias[o] = (heads_early && o < 2 * A) ? (o < A ? a.bm[o] : a.bs[o - A]) : 0.f;
#pragma unroll
    for (int v = 0; v < kHeadRegs / 4; ++v) {
        const int o = (4 * v) / KP, k = (4 * v) % KP;   // (KP is a multiple of 4)
        hw[v] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (heads_early && o < 2 * A)
            hw[v] = *(const f32x4*)((o < A ? a.wm + (size_t)o * H : a.ws + (size_t)(o - A) * H) + p * KP + k);
    }
    // ---- layer 1: h[e][j] = relu(sum_k obs[e][k] W1[j][k] + b1[j]) (k ascending, then the
    // bias): the tile's observations into LDS (h1 is free until the first hidden layer), each
    // thread's columns' weights and biases in registers, all requested together.  SC: S at
    // compile time (the two SAC phases' 2 and 5; 0: any S <= 16, its k loop predicated)
    auto layer1 = [&](auto sc) {
        constexpr int SC = decltype(sc)::value;
        constexpr int KM = SC ? SC : 16;
        const int s1 = SC ? SC : S;
        constexpr int kCols1 = (H + kSacBlock - 1) / kSacBlock;
        float w1[kCols1][KM], b1[kCols1];
#pragma unroll
        for (int c = 0; c < kCols1; ++c) {
            const int j = tid + c * kSacBlock;
#pragma unroll
            for (int k = 0; k < KM; ++k) w1[c][k] = (j < H && k < s1) ? a.w[0][j * s1 + k] : 0.f;
            b1[c] = j < H ? a.b[0][j] : 0.f;
        }
        if (tid < kSacTile * s1) {
            const int te = tid / s1;
            h1[tid] = e0 + te < n ? a.obs[(e0 + te) * s1 + (tid - te * s1)] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < kCols1; ++c) {
            const int j = tid + c * kSacBlock;
            if (j < H) {
#pragma unroll
                for (int te = 0; te < kSacTile; ++te) {
                    float acc = 0.f;
#pragma unroll
                    for (int k = 0; k < KM; ++k) if (k < s1) acc = fmaf(h1[te * s1 + k], w1[c][k], acc);
                    acc += b1[c];
                    h0[te * P + j] = acc < 0.f ? 0.f : acc;
                }
            }
        }
    };
    if (S == 2) layer1(std::integral_constant<int, 2>{});
    else if (S == 5) layer1(std::integral_constant<int, 5>{});
    else layer1(std::integral_constant<int, 0>{});
    __syncthreads();
    mark(0);
    // ---- hidden layers on MFMA: wave w computes the column tiles w, w + 4, ..., NT at a time.
    // The weight fragments go through a wave-private LDS ring by LDS DMA (global_load_lds_dwordx4:
    // a wave instruction moves 1 KB, 8 whole 128-byte row segments, straight into LDS), block
    // kb + 1's transfer in flight while block kb's MFMAs run; chunks are XOR-swizzled by row so
    // that the fragment reads (ds_read_b128, lane (r, q): chunks 2q and 2q + 1 of row r) are free
    // of bank conflicts.
    const int r = lane & 15, q = lane >> 4;
    float* hin = h0;
    float* hout = h1;
    constexpr int kTiles = H / 64;                     // column tiles per wave
    constexpr int NT = kTiles < 2 ? kTiles : 2;        // in flight together
    constexpr int KB = H / 32;                         // k-blocks of 32
    constexpr int kRows = NT * 16;                     // rows of a block (32 floats each)
    float* wring = hb + 2 * kSacTile * P + wave * (2 * kRows * 32);
    for (int l = 1; l < a.L; ++l) {
        const float* W = a.w[l];
#pragma unroll 1
        for (int g = 0; g < kTiles; g += NT) {
            f32x4 acc[NT];
#pragma unroll
            for (int i = 0; i < NT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            // this lane's source in each DMA instruction m (rows 8m .. 8m + 7 of the block)
            auto dma = [&](int kb) {
                float* dst = wring + (kb & 1) * (kRows * 32);
#pragma unroll
                for (int m = 0; m < kRows / 8; ++m) {
                    const int rl = 8 * m + (lane >> 3), i = rl >> 4, rr = rl & 15;
                    const int c = (lane & 7) ^ ((rr >> 1) & 7);
                    const float* src = W + (size_t)(16 * (wave + 4 * (g + i)) + rr) * H + 32 * kb + 4 * c;
                    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(dst + m * 256),
                                                     16, 0, 0);
                }
            };
            dma(0);
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                // block kb's transfer has landed (the only vector-memory operation in flight: the
                // compiler does not order LDS DMA before the LDS reads of its data by itself)
                __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
                __builtin_amdgcn_sched_barrier(0);
                const float* src = wring + (kb & 1) * (kRows * 32);
                f32x4 bf[NT][2];
#pragma unroll
                for (int i = 0; i < NT; ++i)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        bf[i][h] = *(const f32x4*)(src + (16 * i + r) * 32 + 4 * ((2 * q + h) ^ ((r >> 1) & 7)));
                const float* ap = hin + r * P + 32 * kb + 8 * q;
                const f32x4 a0 = *(const f32x4*)ap, a1 = *(const f32x4*)(ap + 4);
                __builtin_amdgcn_sched_barrier(0);
                if (kb + 1 < KB) dma(kb + 1);
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int i = 0; i < NT; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j], bf[i][0][j], acc[i], 0, 0, 0);
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int i = 0; i < NT; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j], bf[i][1][j], acc[i], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);   // (the next block's wait stays behind these MFMAs)
            }
            // D[row 4q + m][col r] + bias, relu, into the next activation tile
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                const int col = 16 * (wave + 4 * (g + i)) + r;
                const float bb = a.b[l][col];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const float v = acc[i][m] + bb;
                    hout[(4 * q + m) * P + col] = v < 0.f ? 0.f : v;
                }
            }
        }
        __syncthreads();
        mark(l);
        float* tmp = hin; hin = hout; hout = tmp;
    }
    // ---- heads: k ascending within a part, a shuffle tree over the 16 parts of each output
    const float* h = hin + e * P + p * KP;
    auto finish = [&](int o, float s, float bias) {
        s += __shfl_xor(s, 8, 16);
        s += __shfl_xor(s, 4, 16);
        s += __shfl_xor(s, 2, 16);
        s += __shfl_xor(s, 1, 16);
        if (p == 0) put(e, o, s + bias);
    };
    if (heads_early) {
        float so[kMaxO];
#pragma unroll
        for (int o = 0; o < kMaxO; ++o) so[o] = 0.f;
#pragma unroll
        for (int v = 0; v < kHeadRegs / 4; ++v) {
            const int o = (4 * v) / KP, k = (4 * v) % KP;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) so[o] = fmaf(h[k + jj], hw[v][jj], so[o]);
        }
#pragma unroll
        for (int o = 0; o < kMaxO; ++o)
            if (o < 2 * A) finish(o, so[o], hb_bias[o]);
    } else {
        for (int o = 0; o < 2 * A; ++o) {
            const float* wr = (o < A ? a.wm + (size_t)o * H : a.ws + (size_t)(o - A) * H) + p * KP;
            float s = 0.f;
#pragma unroll 4
            for (int k = 0; k < KP; ++k) s = fmaf(h[k], wr[k], s);
            finish(o, s, o < A ? a.bm[o] : a.bs[o - A]);
        }
    }
    mark(a.L);
}

}  // namespace pd
