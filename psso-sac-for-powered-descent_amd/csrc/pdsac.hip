// pdsac.hip -- pd_sac_actor: the SAC actor of the c5 collection step as one launch (SURVEY 8f
// rank 3's caller).  The MLP itself (Actor.forward, sac_pytorch.py:129-159: MFMA hidden layers,
// activations in LDS, 16 envs per workgroup) is pd_sac_mlp.h's sac_mlp_tile, which the c5 step
// kernel also runs in its prologue (pd_step_sac_fused: actor + env step in one launch).
#include <hip/hip_runtime.h>

#include "../../include/pdenv.h"
#include "pd_sac_mlp.h"

namespace {

using pd::kSacBlock;
using pd::kSacTile;

template <int H>
__global__ __launch_bounds__(kSacBlock) void k_sac_actor(pd::SacMlp a, int64_t n, float* heads) {
    __shared__ __attribute__((aligned(16))) float hb[pd::sac_mlp_lds_floats<H>()];
    const int64_t e0 = (int64_t)blockIdx.x * kSacTile;
    pd::sac_mlp_tile<H>(a, n, e0, hb, [&](int e, int o, float v) {
        const int64_t ge = e0 + e;
        if (ge < n) heads[ge * 2 * a.A + o] = v;
    });
}

}  // namespace

namespace pd {
pd_status set_error(pd_status s, const char* m);   // pdenv.hip: the pd_last_error() message
}

extern "C" {

pd_status pd_sac_actor(int64_t n, int32_t state_dim, int32_t hidden, int32_t n_hidden_layers, int32_t action_dim,
                       const float* obs, const float* const* params, float* heads, void* stream) {
    if (n < 0 || state_dim < 1 || state_dim > 16 || n_hidden_layers < 1 || n_hidden_layers > pd::kSacMaxLayers ||
        action_dim < 1 || action_dim > 8 || !params || !heads || (n > 0 && !obs))
        return pd::set_error(PD_ERR_INVALID, "pd_sac_actor: bad arguments");
    if (hidden != 128 && hidden != 256 && hidden != 512)
        return pd::set_error(PD_ERR_UNSUPPORTED, "pd_sac_actor: hidden width 128, 256 or 512 only");
    if (n == 0) return PD_OK;
    pd::SacMlp a{};
    a.S = state_dim; a.L = n_hidden_layers; a.A = action_dim; a.H = hidden; a.obs = obs;
    for (int l = 0; l < n_hidden_layers; ++l) {
        a.w[l] = params[2 * l]; a.b[l] = params[2 * l + 1];
        if (!a.w[l] || !a.b[l]) return pd::set_error(PD_ERR_INVALID, "pd_sac_actor: null layer parameter");
    }
    a.wm = params[2 * n_hidden_layers]; a.bm = params[2 * n_hidden_layers + 1];
    a.ws = params[2 * n_hidden_layers + 2]; a.bs = params[2 * n_hidden_layers + 3];
    if (!a.wm || !a.bm || !a.ws || !a.bs) return pd::set_error(PD_ERR_INVALID, "pd_sac_actor: null head parameter");
    // the hidden layers' weights are read as 16-byte vectors (sac_mlp_tile)
    for (int k = 0; k < 2 * (n_hidden_layers + 2); ++k)
        if ((uintptr_t)params[k] % 16 != 0) return pd::set_error(PD_ERR_UNSUPPORTED, "pd_sac_actor: parameter not 16-byte aligned");
    const dim3 grid((unsigned)((n + kSacTile - 1) / kSacTile));
    hipStream_t s = (hipStream_t)stream;
    switch (hidden) {
        case 128: hipLaunchKernelGGL(k_sac_actor<128>, grid, dim3(kSacBlock), 0, s, a, n, heads); break;
        case 512: hipLaunchKernelGGL(k_sac_actor<512>, grid, dim3(kSacBlock), 0, s, a, n, heads); break;
        default: hipLaunchKernelGGL(k_sac_actor<256>, grid, dim3(kSacBlock), 0, s, a, n, heads); break;
    }
    if (hipGetLastError() != hipSuccess) return pd::set_error(PD_ERR_HIP, "pd_sac_actor: launch failed");
    return PD_OK;
}

}  // extern "C"
