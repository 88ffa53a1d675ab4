"""The stochastic draws of the device against the reference's DISTRIBUTIONS.

The reference cannot be replayed (np.random.seed(None), vonkarman.py:88), so the per-step parity
tests pin the device to the oracle's restatement of the device's own Philox scheme.  These tests
tie that scheme to what the reference draws, on the device, through the product path:

- per reset, VKDisturbanceGenerator._new_filters (vonkarman.py:60-66): sigma_u ~ U(0.5, 2.25),
  sigma_v ~ U(1.25, 2.0);
- per reset, WindModel(given_percentile=None) (full_wind_model.py:27-33):
  percentile = np.random.randint(50, 99), uniform on 50..98, never 99;
- per reset, the pitch tilt of the c3 configuration: theta += N(0, 1 deg);
- per filter step, vonkarman.py:34: one np.random.randn() for u, one for v: N(0, 1);
- the reference draws these from separate np.random calls: independent.

Tests: Kolmogorov-Smirnov for the continuous laws, chi-square for the percentile and for the
independence of the percentile and the sigmas.  With fixed seeds the p-values are fixed numbers;
the bound p > 1e-4 fails a range, modulo or correlation defect (p ~ 0) without being flaky.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
P_MIN = 1e-4


@pytest.fixture(scope="module")
def pd():
    import torch
    import pdenv
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return pdenv


def _reset_samples(pd, n=65536, resets=2, seed=1234):
    """(sigma_u, sigma_v, percentile, tilt in degrees) of `resets` x n in-library resets (k_reset)."""
    env = pd.PoweredDescentEnv(n, flight_phase="landing_burn_pure_throttle", mode="rl", enable_wind=True,
                               stochastic_wind=True, wind_percentile=None, auto_reset=True,
                               tilt_sigma_rad=math.radians(1.0), seed=seed)
    th0 = env.params.state0[4]
    su, sv, pr, tilt = [], [], [], []
    for _ in range(resets):
        env.reset()
        _, sig, p = env.wind_state()
        s = env.state
        su.append(sig[:, 0].cpu().numpy()); sv.append(sig[:, 1].cpu().numpy()); pr.append(p.cpu().numpy())
        tilt.append(np.degrees(s[:, 4].cpu().numpy() - th0))
        # alpha = theta - gamma after the tilt
        assert np.array_equal(s[:, 7].cpu().numpy(), (s[:, 4] - s[:, 6]).cpu().numpy())
    ep, _, _ = env.episode_counters()
    assert int(ep.min()) == int(ep.max()) == resets     # every env drew `resets` distinct episodes
    env.close()
    return (np.concatenate(su), np.concatenate(sv), np.concatenate(pr), np.concatenate(tilt))


def test_reset_draw_distributions(pd):
    """131 072 resets: sigma_u ~ U(0.5, 2.25), sigma_v ~ U(1.25, 2.0) (KS), the percentile
    uniform on 50..98 (chi-square, 49 cells, 99 never drawn), the tilt ~ N(0, 1 deg) (KS)."""
    from scipy import stats
    su, sv, pr, tilt = _reset_samples(pd)
    assert su.min() >= 0.5 and su.max() < 2.25 and sv.min() >= 1.25 and sv.max() < 2.0
    assert stats.kstest(su, stats.uniform(0.5, 1.75).cdf).pvalue > P_MIN
    assert stats.kstest(sv, stats.uniform(1.25, 0.75).cdf).pvalue > P_MIN
    assert pr.min() == 50 and pr.max() == 98, (pr.min(), pr.max())
    counts = np.bincount(pr - 50, minlength=49)
    assert len(counts) == 49 and counts.min() > 0
    assert stats.chisquare(counts).pvalue > P_MIN
    assert stats.kstest(tilt, stats.norm(0.0, 1.0).cdf).pvalue > P_MIN
    assert abs(tilt.mean()) < 5 / math.sqrt(len(tilt)) and abs(tilt.std() - 1.0) < 0.01


def test_reset_draws_independent(pd):
    """The percentile is independent of sigma_u and sigma_v, and sigma_u of sigma_v (chi-square
    contingency over 7 percentile groups x 8 sigma bins; round 2 drew the percentile from the
    sigmas' own Philox words).  The tilt is independent of the percentile."""
    from scipy import stats
    su, sv, pr, tilt = _reset_samples(pd, seed=77)
    grp = (pr - 50) // 7                                     # 7 groups of 7 percentiles
    for x, lo, hi in ((su, 0.5, 2.25), (sv, 1.25, 2.0)):
        b = np.minimum(((x - lo) / (hi - lo) * 8).astype(int), 7)
        tab = np.zeros((7, 8), dtype=np.int64)
        np.add.at(tab, (grp, b), 1)
        assert stats.chi2_contingency(tab).pvalue > P_MIN
    bu = np.minimum(((su - 0.5) / 1.75 * 8).astype(int), 7)
    bv = np.minimum(((sv - 1.25) / 0.75 * 8).astype(int), 7)
    tab = np.zeros((8, 8), dtype=np.int64)
    np.add.at(tab, (bu, bv), 1)
    assert stats.chi2_contingency(tab).pvalue > P_MIN
    bt = np.clip(np.floor(tilt + 2).astype(int), 0, 3)       # tilt quartile-ish bins in degrees
    tab = np.zeros((7, 4), dtype=np.int64)
    np.add.at(tab, (grp, bt), 1)
    assert stats.chi2_contingency(tab).pvalue > P_MIN


def test_gust_normals_distribution(pd):
    """>= 1e6 gust normals drawn by k_step's wind block (vonkarman.py:34), recovered exactly:
    a phase with one physics call per env step (landing_burn_pure_throttle_Pcontrol) inside the
    gust band, the filter states zeroed before each step, so that after it
    f_u = (0 + 0) + (sigma_u Bd_u[0]) w_u (vonkarman.py:33-36) and w_u = f_u / (sigma_u Bd_u[0]).
    KS against N(0, 1), the first four moments, and u/v independence."""
    import torch
    from scipy import stats
    N, T = 65536, 8
    env = pd.PoweredDescentEnv(N, flight_phase="landing_burn_pure_throttle_Pcontrol", mode="rl", enable_wind=True,
                               stochastic_wind=True, wind_percentile=50, auto_reset=False, seed=4321)
    S = env.state
    S[:, 1] = 10000.0                                        # below the 15 km gust ceiling
    env.set_state(S)
    P = env.params.struct
    bu0, bu1, bv0, bv1 = P.vk_Bd_u[0], P.vk_Bd_u[1], P.vk_Bd_v[0], P.vk_Bd_v[1]
    _, sig, _ = env.wind_state()
    zeros = torch.zeros(N, 4, dtype=torch.float64, device="cuda")
    act = torch.zeros(N, 1, dtype=torch.float32, device="cuda")
    wu, wv = [], []
    for _ in range(T):
        env.set_wind_state(filters=zeros)
        env.step(act)
        f, _, _ = env.wind_state()
        assert bool((env.state[:, 1] < 15000.0).all())
        u = f[:, 0] / (sig[:, 0] * bu0)
        v = f[:, 2] / (sig[:, 1] * bv0)
        # the second filter component carries the same normal (Bd's second entry)
        assert torch.allclose(f[:, 1], (sig[:, 0] * bu1) * u, rtol=1e-12, atol=0)
        assert torch.allclose(f[:, 3], (sig[:, 1] * bv1) * v, rtol=1e-12, atol=0)
        wu.append(u.cpu().numpy()); wv.append(v.cpu().numpy())
    wu, wv = np.concatenate(wu), np.concatenate(wv)
    w = np.concatenate([wu, wv])
    assert len(w) >= 1_000_000
    assert len(np.unique(w)) == len(w)                       # no repeated Philox counter
    assert stats.kstest(w, stats.norm.cdf).pvalue > P_MIN
    n = len(w)
    assert abs(w.mean()) < 5 / math.sqrt(n)
    assert abs(w.var() - 1.0) < 5 * math.sqrt(2.0 / n)
    assert abs(stats.skew(w)) < 5 * math.sqrt(6.0 / n)
    assert abs(stats.kurtosis(w)) < 5 * math.sqrt(24.0 / n)
    assert abs(np.corrcoef(wu, wv)[0, 1]) < 5 / math.sqrt(len(wu))
    env.close()
