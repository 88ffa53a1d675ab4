import os, sys, numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "psso-sac-for-powered-descent_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import pdenv, oracle
for lpe in (1, 4):
    for ar in (False, True):
        N = 4096
        env = pdenv.PoweredDescentEnv(N, mode="rl", auto_reset=ar, lanes_per_env=lpe)
        rng = np.random.default_rng(0)
        A = rng.uniform(-1, 1, (200, N, 1)).astype(np.float32)
        ends = []
        for t in range(200):
            obs, r, dn, tr, ex = env.step(torch.from_numpy(A[t]).cuda())
            ends.append(int((dn | tr).sum()))
        tid = ex["trunc_id"].cpu().numpy()
        print("lpe", lpe, "auto_reset", ar, "first end step", next((i for i, e in enumerate(ends) if e), None),
              "total ends", sum(ends), "tid hist", np.bincount(tid.astype(np.int64) + 0, minlength=9))
        o = oracle.Oracle(0, 0)
        for t in range(200):
            s, rr, d_, tr_, tid_, ob, info = o.step(A[t, 0], True)
            if d_ or tr_:
                print("   oracle env0 ends at", t, tid_); break
