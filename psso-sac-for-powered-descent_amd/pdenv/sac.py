"""SAC data path on the device (SURVEY config c5): the reference's actor drives N envs per GPU,
transitions are all-gathered over RCCL into a device replay buffer on the learner rank.

The reference steps ONE env per process and adds one transition per step to a numpy buffer
(sac_pytorch_powered_descent.py:160-183, sac_pytorch.py:12-49).  Here every rank steps its own
env shard through libpdenv, builds the transition slab [n_local, s|a|r|s'|done] (28 B per env
for the pure-throttle task), and `all_gather_into_tensor` (backend "nccl" = RCCL over xGMI)
concatenates the slabs in rank order; the learner rank appends them to its ring buffer.  The
learner itself (critic/actor updates) is the caller's, as in the reference.
"""
import ctypes as C

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L
from .env import _ptr, _stream


class Actor(nn.Module):
    """sac_pytorch.py:129-179: shared MLP (ReLU), mean and log_std heads, tanh squashing."""

    def __init__(self, state_dim, action_dim, hidden_dim=256, n_hidden_layers=2, max_action=1.0,
                 log_std_min=-20.0, log_std_max=2.0):
        super().__init__()
        self.max_action, self.log_std_min, self.log_std_max = max_action, log_std_min, log_std_max
        layers = [nn.Linear(state_dim, hidden_dim), nn.ReLU()]
        for _ in range(n_hidden_layers - 1):
            layers += [nn.Linear(hidden_dim, hidden_dim), nn.ReLU()]
        self.shared_net = nn.Sequential(*layers)
        self.mean = nn.Linear(hidden_dim, action_dim)
        self.log_std = nn.Linear(hidden_dim, action_dim)

    def forward(self, state):
        f = self.shared_net(state)
        return self.mean(f), torch.clamp(self.log_std(f), self.log_std_min, self.log_std_max)

    def sample(self, state, deterministic=False, generator=None, with_log_prob=True):
        """with_log_prob=False skips the log-probability (select_action discards it,
        sac_pytorch_powered_descent.py / sac_pytorch.py:404-409): same action, fewer kernels."""
        mean, log_std = self(state)
        if deterministic:
            return torch.tanh(mean) * self.max_action, None
        std = log_std.exp()
        eps = torch.randn(mean.shape, device=mean.device, dtype=mean.dtype, generator=generator)
        x = mean + std * eps                                   # Normal(mean, std).rsample()
        action = torch.tanh(x)
        if not with_log_prob:
            return action * self.max_action, None
        log_prob = (-((x - mean) ** 2) / (2 * std ** 2) - log_std - 0.9189385332046727
                    - torch.log(1 - action.pow(2) + 1e-6)).sum(-1, keepdim=True)
        return action * self.max_action, log_prob


class DeviceReplayBuffer:
    """The reference's uniform ReplayBuffer (sac_pytorch.py:12-49) as device tensors.
    add_batch appends B transitions at once (ring, oldest overwritten)."""

    def __init__(self, capacity, state_dim, action_dim, device):
        self.capacity, self.state_dim, self.action_dim = int(capacity), state_dim, action_dim
        self.width = 2 * state_dim + action_dim + 2
        self.data = torch.zeros(self.capacity, self.width, dtype=torch.float32, device=device)
        self.position = 0
        self.size = 0
        # the ring's position and size on the device (int64: position, size, pd_step_sac_ring's
        # workgroup counter): the collection kernel writes its rows there and advances them, the
        # host mirrors (position, size) by note_appended
        self.state_dev = torch.zeros(3, dtype=torch.int64, device=device)

    def _sync_state_dev(self):
        # device-side fills (no host tensor, so no blocking pageable copy on the step's stream)
        self.state_dev[0].fill_(self.position)
        self.state_dev[1].fill_(self.size)
        self.state_dev[2].zero_()

    def note_appended(self, b):
        """The host mirror of b rows appended on the device (pd_step_sac_ring)."""
        self.position = (self.position + b) % self.capacity
        self.size = min(self.size + b, self.capacity)

    def rows(self, start, b):
        """The b ring rows from start (a view unless they wrap)."""
        end = start + b
        if end <= self.capacity:
            return self.data[start:end]
        return torch.cat([self.data[start:], self.data[:end - self.capacity]])

    def add_batch(self, slab):
        """slab [B, 2S + A + 2] = state | action | reward | next_state | done (float32)."""
        b = slab.shape[0]
        if b > self.capacity:
            slab, b = slab[-self.capacity:], self.capacity
        end = self.position + b
        if end <= self.capacity:
            self.data[self.position:end] = slab
        else:
            k = self.capacity - self.position
            self.data[self.position:] = slab[:k]
            self.data[:b - k] = slab[k:]
        self.position = end % self.capacity
        self.size = min(self.size + b, self.capacity)
        self._sync_state_dev()

    def add(self, state, action, reward, next_state, done):
        """The reference's one-transition add (sac_pytorch.py:27-35)."""
        row = torch.cat([torch.as_tensor(state, dtype=torch.float32).reshape(-1),
                         torch.as_tensor(action, dtype=torch.float32).reshape(-1),
                         torch.tensor([float(reward)]),
                         torch.as_tensor(next_state, dtype=torch.float32).reshape(-1),
                         torch.tensor([float(done)])]).to(self.data.device)
        self.add_batch(row[None])

    def sample(self, batch_size, generator=None):
        """Uniform indices in [0, size) (np.random.randint, sac_pytorch.py:37-46)."""
        idx = torch.randint(0, self.size, (batch_size,), device=self.data.device, generator=generator)
        d = self.data[idx]
        S, A = self.state_dim, self.action_dim
        return (d[:, :S], d[:, S:S + A], d[:, S + A:S + A + 1], d[:, S + A + 1:2 * S + A + 1],
                d[:, 2 * S + A + 1:])

    def __len__(self):
        return self.size


class DevicePrioritizedReplayBuffer(DeviceReplayBuffer):
    """The reference's PrioritizedReplayBuffer (sac_pytorch.py:51-127; the SAC driver's buffer,
    use_per=True) as device tensors.

    New transitions get the current max priority.  sample() draws batch_size distinct indices
    with probability proportional to priority**alpha without replacement -- the distribution of
    np.random.choice(size, batch, replace=False, p=probs) -- by the Gumbel-top-k construction
    (top-k of alpha*log(priority) + Gumbel noise), returns importance weights
    (size*probs)**(-beta) / max, and anneals beta."""

    def __init__(self, capacity, state_dim, action_dim, device, alpha=0.6, beta=0.4,
                 beta_annealing_steps=100000, epsilon=1e-6):
        super().__init__(capacity, state_dim, action_dim, device)
        self.alpha, self.beta, self.epsilon = alpha, beta, epsilon
        self.beta_increment = (1.0 - beta) / beta_annealing_steps
        self.priorities = torch.zeros(self.capacity, dtype=torch.float32, device=device)
        self.max_priority = 1.0
        self.max_prio_dev = torch.ones(1, dtype=torch.float32, device=device)   # (read by pd_step_sac_ring)

    def add_batch(self, slab):
        b = min(slab.shape[0], self.capacity)
        if self.position + b <= self.capacity:                 # no wrap: one fill
            self.priorities[self.position:self.position + b] = self.max_priority
        else:                                                  # wrap: the tail, then the head
            k = self.capacity - self.position
            self.priorities[self.position:] = self.max_priority
            self.priorities[:b - k] = self.max_priority
        super().add_batch(slab)

    def sample(self, batch_size, generator=None):
        if self.size == 0:
            return None
        pr = self.priorities[:self.size].double()
        probs = pr ** self.alpha
        probs = probs / probs.sum()
        u = torch.rand(self.size, dtype=torch.float64, device=self.data.device, generator=generator)
        gumbel = -torch.log(-torch.log(u.clamp_min(1e-300)))
        idx = torch.topk(torch.log(probs) + gumbel, batch_size).indices
        w = (self.size * probs[idx]) ** (-self.beta)
        w = (w / w.max()).float().reshape(-1, 1)
        self.beta = min(1.0, self.beta + self.beta_increment)
        d = self.data[idx]
        S, A = self.state_dim, self.action_dim
        return (d[:, :S], d[:, S:S + A], d[:, S + A:S + A + 1], d[:, S + A + 1:2 * S + A + 1],
                d[:, 2 * S + A + 1:], w, idx)

    def update_priorities(self, indices, td_errors):
        """sac_pytorch.py:120-124: priority = |td| + epsilon; max_priority tracks the largest."""
        p = td_errors.detach().reshape(-1).abs().float() + self.epsilon
        self.priorities[indices] = p
        self.max_priority = max(self.max_priority, float(p.max()))
        self.max_prio_dev.fill_(self.max_priority)


def transition_slab(obs, action, reward, next_obs, done):
    """[N, 2S + A + 2] float32: state | action | reward | next_state | done (done, not truncated,
    as the driver stores it: sac_pytorch_powered_descent.py:170-176)."""
    return torch.cat([obs.float(), action.float(), reward.float()[:, None], next_obs.float(),
                      done.float()[:, None]], dim=1).contiguous()


def gather_slabs(slab, dist=None):
    """All ranks' slabs concatenated in rank order (all_gather_into_tensor; RCCL on GPU ranks)."""
    if dist is None or not dist.is_initialized():
        return slab
    out = torch.empty((dist.get_world_size() * slab.shape[0], slab.shape[1]), dtype=slab.dtype,
                      device=slab.device)
    dist.all_gather_into_tensor(out, slab)
    return out


class ActorKernel:
    """The Actor's forward pass as one pd_sac_actor launch (the shared MLP on MFMA and both heads,
    activations in LDS): obs [N, S] float32 -> heads [N, 2A] (mean | log_std, unclamped).  Reads
    the actor's parameter tensors in place (no copies: an optimizer step or an in-place update of
    any kind is seen by the next call; a captured graph keeps the parameter addresses it saw, so
    replacing a parameter tensor -- `.data = ...` -- needs a re-capture).  supported(actor) tells
    whether the shapes fit the kernel (hidden 128/256/512, <= 8 hidden layers, S <= 16, A <= 8,
    float32 parameters on the device)."""

    def __init__(self, actor):
        self.actor = actor
        self.lib = L.load()
        lins = [m for m in actor.shared_net if isinstance(m, nn.Linear)]
        self.S, self.H, self.A = lins[0].in_features, lins[0].out_features, actor.mean.out_features
        self.nl = len(lins)
        self.params = [t for m in lins for t in (m.weight, m.bias)] + [actor.mean.weight, actor.mean.bias,
                                                                       actor.log_std.weight, actor.log_std.bias]
        self._ptrs = (C.c_void_p * len(self.params))()

    @staticmethod
    def supported(actor):
        lins = [m for m in actor.shared_net if isinstance(m, nn.Linear)]
        acts = [m for m in actor.shared_net if not isinstance(m, nn.Linear)]
        if not lins or len(lins) > 8 or any(not isinstance(m, nn.ReLU) for m in acts) or len(acts) != len(lins):
            return False
        H = lins[0].out_features
        ps = [p for m in lins for p in (m.weight, m.bias)] + list(actor.mean.parameters()) + list(actor.log_std.parameters())
        return (H in (128, 256, 512) and lins[0].in_features <= 16 and actor.mean.out_features <= 8
                and all(m.in_features == H and m.out_features == H for m in lins[1:])
                and all(p.dtype == torch.float32 and p.is_cuda and p.is_contiguous() and p.data_ptr() % 16 == 0
                        for p in ps))

    def ptrs(self):
        """The parameter pointers as pd_sac_actor / pd_step_sac_fused take them (read now: an
        in-place update keeps them, a replaced tensor is picked up here)."""
        for k, t in enumerate(self.params):
            self._ptrs[k] = t.data_ptr()
        return self._ptrs

    def __call__(self, obs, heads):
        L.check(self.lib.pd_sac_actor(int(obs.shape[0]), self.S, self.H, self.nl, self.A, _ptr(obs), self.ptrs(),
                                      _ptr(heads), _stream(obs.device)))
        return heads


class SACCollector:
    """One collection step of N envs on this rank: actor -> env step -> transition rows -> (gather)
    -> learner-rank buffer.  `obs` always holds the observation the actor sees next (the
    post-auto-reset observation of envs whose episode ended).

    fused=True (default): ONE launch per step where the actor fits the kernel (ActorKernel
    shapes; pd_step_sac_fused): the reference Actor's MLP and both heads for each workgroup's 16
    envs in the step kernel's prologue (MFMA hidden layers, activations in LDS), then the action
    sampled from the heads (eps drawn there, Philox; torch.randn's role), the env step, and the
    transition rows written by the kernel epilogue straight into the learner's replay ring at the
    ring's device-held position, with the new rows' priorities set to the buffer's max priority;
    the next float32 observation into `obs`.  (Handles that do not step 16 lanes per env: the
    actor as its own launch, pd_sac_actor, the same bits.)  Actor shapes the kernel does not
    cover: PyTorch's shared_net and one GEMM over both heads, then pd_step_sac_ring.  On several
    ranks the rows go to a local slab instead and `all_gather_into_tensor` (RCCL) appends them
    on the learner rank.
    fused=False: Actor.sample, pd_step, transition_slab, pd_observe, buffer.add_batch (the unfused
    reference path, eps from torch.randn with `generator`).
    use_graph=True captures the step into one HIP graph (the ring position lives on the device, so
    replays append in order).  Off by default: on ROCm 7 each replay of the one-kernel graph left
    an 8.6 us gap before its step kernel, where eager launches from a host that keeps ahead of
    the GPU run back to back (c5: 0.0434 against 0.0392 ms per step, profiles/r05_exp_c5_graph.jsonl).  The gather runs eagerly after
    each replay.  flush_every > 0: a pd_flush_misses call every that many steps (0, the default:
    none -- the step launch inserts the neighbourhoods it solved itself, ABI 10).
    step() returns the step's transition rows: a view of the replay ring's rows (valid until the
    ring wraps onto them) in ring mode, else a fresh tensor."""

    def __init__(self, env, actor, buffer=None, dist=None, learner_rank=0, generator=None,
                 deterministic=False, use_graph=False, flush_every=0, fused=True):
        self.env, self.actor, self.buffer, self.dist = env, actor, buffer, dist
        self.learner_rank, self.generator, self.deterministic = learner_rank, generator, deterministic
        self.rank = dist.get_rank() if dist is not None and dist.is_initialized() else 0
        self.multi = dist is not None and dist.is_initialized() and dist.get_world_size() > 1
        self.obs = env.reset().float().contiguous()
        self.flush_every = flush_every
        self.steps = 0
        self.graph = None
        self.use_graph = use_graph
        self.fused = fused
        S, A = env.obs_dim, env.action_dim
        dev = self.obs.device
        self._slab_buf = torch.empty(env.n, 2 * S + A + 2, dtype=torch.float32, device=dev)
        self.action = torch.empty(env.n, A, dtype=torch.float32, device=dev)
        self.heads = torch.empty(env.n, 2 * A, dtype=torch.float32, device=dev)
        self.eps_out = None           # [N, A] to receive the kernel's eps draws (tests)
        self.heads_out = None         # [N, 2A] to receive the actor's heads (tests)
        self.kernel = ActorKernel(actor) if fused and ActorKernel.supported(actor) else None
        H = actor.mean.in_features
        self._head_w = torch.empty(2 * A, H, dtype=torch.float32, device=dev)
        self._head_b = torch.empty(2 * A, dtype=torch.float32, device=dev)
        # ring mode: this process holds the buffer and steps every env of the job
        self.ring = fused and buffer is not None and not self.multi and buffer.capacity >= env.n

    def _heads(self):
        if self.kernel is not None:
            return self.kernel(self.obs, self.heads)
        # (shapes pd_sac_actor does not cover) torch's MLP and one GEMM over both heads, the
        # head weights copied on every step (inside a captured graph too: never stale)
        a = self.actor
        torch.cat([a.mean.weight, a.log_std.weight], out=self._head_w)
        torch.cat([a.mean.bias, a.log_std.bias], out=self._head_b)
        f = a.shared_net(self.obs)
        return torch.addmm(self._head_b, f, self._head_w.t(), out=self.heads)

    def _body(self):
        """actor -> env step -> transition rows and next obs into self.obs (no syncs); returns
        the local slab, or None when the rows went straight into the replay ring."""
        if self.fused:
            a = self.actor
            kw = dict(deterministic=self.deterministic, action=self.action, obs32=self.obs, eps_out=self.eps_out)
            if self.ring:
                b = self.buffer
                kw.update(ring=b.data, capacity=b.capacity, ring_state=b.state_dev,
                          priorities=getattr(b, "priorities", None), max_priority=getattr(b, "max_prio_dev", None))
            else:
                kw.update(ring=self._slab_buf)
            if self.kernel is not None:
                k = self.kernel
                self.env.step_sac_fused(k.S, k.A, k.H, k.nl, k.ptrs(), a.log_std_min, a.log_std_max, a.max_action,
                                        heads=self.heads_out, **kw)
            else:
                self.env.step_sac_ring(self._heads(), a.log_std_min, a.log_std_max, a.max_action, **kw)
            return None if self.ring else self._slab_buf
        gen = None if self.use_graph else self.generator
        act, _ = self.actor.sample(self.obs, deterministic=self.deterministic, generator=gen, with_log_prob=False)
        act = act.float().contiguous()
        self.env.step_raw_noflush(act)
        slab = transition_slab(self.obs, act, self.env.reward_buf, self.env.obs_buf, self.env.done_buf)
        self.obs.copy_(self.env.observe_raw())                 # copy_ casts: one kernel
        return slab

    def _finish(self, slab):
        self.steps += 1
        if self.flush_every and self.steps % self.flush_every == 0:
            self.env.flush()
        if slab is None:                                       # ring mode: the rows are in place
            start = self.buffer.position
            self.buffer.note_appended(self.env.n)
            return self.buffer.rows(start, self.env.n)
        full = gather_slabs(slab, self.dist)
        if self.rank == self.learner_rank and self.buffer is not None:
            self.buffer.add_batch(full)
        return full.clone() if full is self._slab_buf else full

    @torch.no_grad()
    def step(self):
        if not self.use_graph:
            return self._finish(self._body())
        if self.graph is None:
            # one eager step on a side stream warms the allocator and the kernels; it is a real
            # step (its transitions are kept), then the next step is captured and replayed
            s = torch.cuda.Stream(device=self.obs.device)
            s.wait_stream(torch.cuda.current_stream(self.obs.device))
            with torch.cuda.stream(s):
                slab = self._body()
            torch.cuda.current_stream(self.obs.device).wait_stream(s)
            full = self._finish(slab)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._slab = self._body()
            return full
        self.graph.replay()
        return self._finish(self._slab)
