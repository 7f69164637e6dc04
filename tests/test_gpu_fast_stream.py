"""The opt-in fast demand stream (demand_stream="philox", include/invsim.h
INVSIM_DEMAND_PHILOX): rocRAND Philox4x32-10 used counter-based with numpy's
PTRS / multiplication transforms.  It is NOT the reference's stream, so parity
is replaced by statistics: a chi-square goodness-of-fit against the Poisson
pmf over >= 1e8 draws per rate (both sampler branches and the boundary
lam = 10), plus the stream's own contracts (opt-in, rollout == steps,
checkpoint round trip, the PCG64 states untouched)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_fast_stream_is_opt_in(gpu):
    import invsim
    env = invsim.InvManagementBacklogEnv(256, device=gpu, record_demand=True)
    assert env.demand_stream == "numpy"
    env.reset(seed=3)
    a = torch.full((256, 3), 10, dtype=torch.int64, device=gpu)
    d_np = env.step(a)[4]["demand"].clone()
    env2 = invsim.InvManagementBacklogEnv(256, device=gpu, record_demand=True, demand_stream="philox")
    assert env2.demand_stream == "philox"
    env2.reset(seed=3)
    d_ph = env2.step(a)[4]["demand"].clone()
    assert not torch.equal(d_np, d_ph)
    with pytest.raises(ValueError):
        env.set_demand_stream("rocrand-xorwow")


def _chi2_poisson(counts, lam, n):
    from scipy.stats import chi2, poisson
    k = np.arange(len(counts))
    p = poisson.pmf(k, lam)
    p[-1] += poisson.sf(len(counts) - 1, lam)         # the last bin takes the upper tail
    exp = p * n
    # pool bins with expected count < 50 into their neighbours (both tails)
    obs_b, exp_b = [], []
    o_acc = e_acc = 0.0
    for o, e in zip(counts, exp):
        o_acc += o
        e_acc += e
        if e_acc >= 50:
            obs_b.append(o_acc)
            exp_b.append(e_acc)
            o_acc = e_acc = 0.0
    if e_acc > 0:
        obs_b[-1] += o_acc
        exp_b[-1] += e_acc
    obs_b, exp_b = np.array(obs_b), np.array(exp_b)
    stat = float(((obs_b - exp_b) ** 2 / exp_b).sum())
    dof = len(obs_b) - 1
    return stat, dof, float(chi2.sf(stat, dof))


@pytest.mark.parametrize("lam", [0.3, 5.0, 9.99, 10.0, 20.0, 162.65])
def test_fast_stream_poisson_chi_square_1e8(gpu, lam):
    import invsim
    n, cycles = 65536, 51                        # 51 episodes x 30 draws x 65 536 envs = 1.003e8
    env = invsim.InvManagementLostSalesEnv(n, device=gpu, dist_param={"mu": lam}, record_demand=True,
                                           demand_stream="philox", copy=False)
    env.reset(seed=11)
    a = torch.zeros((n, 3), dtype=torch.int64, device=gpu)
    hi = int(lam + 12 * np.sqrt(lam) + 30)
    counts = torch.zeros(hi + 1, dtype=torch.int64, device=gpu)
    s1 = torch.zeros((), dtype=torch.float64, device=gpu)
    lag = torch.zeros((), dtype=torch.float64, device=gpu)
    prev = None
    draws = 0
    for k in range(31 * cycles):
        _, _, _, tr, info = env.step(a)
        if k % 31 == 30:                         # the NEXT_STEP reset call draws nothing
            prev = None
            continue
        d = info["demand"]
        counts += torch.bincount(d.clamp(max=hi), minlength=hi + 1)
        s1 += d.sum(dtype=torch.float64)
        if prev is not None:
            lag += (d.double() * prev.double()).sum()
        prev = d
        draws += n
    assert draws >= 100_000_000
    c = counts.cpu().numpy().astype(np.float64)
    stat, dof, p = _chi2_poisson(c, lam, draws)
    assert p > 1e-4, f"chi-square {stat:.1f} on {dof} dof, p = {p:.2e}"
    mean = float(s1) / draws
    assert abs(mean - lam) < 6 * np.sqrt(lam / draws)
    # consecutive steps of an env are uncorrelated: E[d_t d_t+1] = lam^2
    pairs = (31 - 2) * cycles * n
    assert abs(float(lag) / pairs - lam * lam) < 6 * lam * np.sqrt((1 + 2 * lam) / pairs) + 1e-12


def test_fast_stream_rollout_equals_steps_and_keeps_pcg_states(gpu):
    import invsim
    n, K = 4096, 70
    mk = lambda: invsim.InvManagementBacklogEnv(n, device=gpu, demand_stream="philox")  # noqa: E731
    e1, e2 = mk(), mk()
    e1.reset(seed=5)
    e2.reset(seed=5)
    rng0 = e1.state_fields()["rng"].clone()
    g = torch.Generator(device=gpu)
    g.manual_seed(1)
    acts = torch.randint(0, 90, (K, n, 3), device=gpu, generator=g)
    o1, r1, _, t1 = e1.rollout(acts)
    for k in range(K):
        o, r, _, t, _ = e2.step(acts[k])
        assert torch.equal(o, o1[k]) and torch.equal(r, r1[k]) and torch.equal(t, t1[k]), k
    assert torch.equal(e1.state_fields()["rng"], rng0)          # the parity stream is untouched


@pytest.mark.parametrize("cls", ["NewsvendorEnv", "NetInvMgmtBacklogEnv", "InvManagementBacklogEnv"])
def test_fast_stream_checkpoint_round_trip(gpu, cls):
    import invsim
    n = 1000
    env = getattr(invsim, cls)(n, device=gpu, demand_stream="philox")
    env.reset(seed=9)
    A = env.action_dim
    dt = env.act_dtype
    a = (torch.ones((n, A), device=gpu) * 20).to(dt)
    for _ in range(7):
        env.step(a)
    blob = env.get_state().clone()
    ref = [env.step(a)[:2] for _ in range(40)]
    env2 = getattr(invsim, cls)(n, device=gpu, demand_stream="philox")
    env2.set_state(blob)
    for k in range(40):
        o, r = env2.step(a)[:2]
        assert torch.equal(o, ref[k][0]) and torch.equal(r.view(torch.int64), ref[k][1].view(torch.int64)), k


def test_fast_stream_newsvendor_and_net_rates(gpu):
    """Newsvendor: demand ~ Poisson(mu) with mu ~ U(0, mu_max) per episode, so
    E[d] = mu_max / 2; Net default graph: one market, Poisson(20)."""
    import invsim
    n = 65536
    nv = invsim.NewsvendorEnv(n, device=gpu, record_demand=True, demand_stream="philox")
    nv.reset(seed=1)
    a = torch.zeros((n, 1), device=gpu)
    tot, cnt = 0.0, 0
    for k in range(41 * 4):
        d = nv.step(a)[4]["demand"]
        if k % 41 != 40:
            tot += float(d.sum())
            cnt += n
    assert abs(tot / cnt - 100.0) < 1.0
    net = invsim.NetInvMgmtBacklogEnv(32768, device=gpu, record_demand=True, demand_stream="philox")
    net.reset(seed=2)
    a = torch.zeros((32768, net.action_dim), device=gpu)
    ds = torch.stack([net.step(a)[4]["demand"].double() for _ in range(30)])
    assert abs(float(ds.mean()) - 20.0) < 0.05
    assert abs(float(ds.var()) - 20.0) < 0.5


def _im_fast_run(gpu, cls, n, fused, monkeypatch, **kw):
    import invsim
    for v in ("INVSIM_IM_SPLIT", "INVSIM_IM_ROLL", "INVSIM_IM_POL_ROLL"):
        monkeypatch.setenv(v, "1" if fused else "0")
    env = getattr(invsim, cls)(n, device=gpu, demand_stream="philox", record_demand=True, **kw)
    env.reset(seed=17)
    g = torch.Generator(device=gpu)
    g.manual_seed(4)
    out = []
    for k in range(33):                                   # split steps, across the NEXT_STEP reset
        a = torch.randint(0, 120, (n, 3), device=gpu, generator=g)
        o, r, te, tr, info = env.step(a)
        out += [o.clone(), r.clone(), tr.clone(), info["demand"].clone()]
    acts = torch.randint(0, 120, (45, n, 3), device=gpu, generator=g)
    out += list(env.rollout(acts))                         # fused rollout
    m = torch.zeros((n, 6), dtype=torch.float64, device=gpu)
    pol = env.rollout_policy(invsim.BaseStockAgent(1.1), 40, obs=True, actions=True, metrics=m)
    out += [pol[k] for k in sorted(pol)] + [m]
    out.append(env.get_state())
    return out


@pytest.mark.parametrize("cls", ["InvManagementBacklogEnv", "InvManagementLostSalesEnv"])
@pytest.mark.parametrize("n", [4096, 65536])
def test_fast_stream_fused_kernels_equal_run_kernel(gpu, monkeypatch, cls, n):
    """The fast stream on the split step kernel and the 2-/3-role rollout
    kernels (no lookahead: draws at (key, launch step)) gives the one-wave run
    kernel's results bit for bit: steps, rollouts, policy rollouts, demands and
    the state blob."""
    a = _im_fast_run(gpu, cls, n, True, monkeypatch)
    b = _im_fast_run(gpu, cls, n, False, monkeypatch)
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x.view(torch.uint8) if x.dtype == torch.float64 else x,
                           y.view(torch.uint8) if y.dtype == torch.float64 else y), i


@pytest.mark.parametrize("dist,param", [(2, {"n": 40, "p": 0.45}), (3, {"low": 3, "high": 37})])
def test_fast_stream_split_numpy_samplers_equal_run_kernel(gpu, monkeypatch, dist, param):
    """Binomial / integers demand (the u32 half not carried on the fast stream)
    on the split step kernel == the run kernel."""
    a = _im_fast_run(gpu, "InvManagementBacklogEnv", 3000, True, monkeypatch, dist=dist, dist_param=param)
    b = _im_fast_run(gpu, "InvManagementBacklogEnv", 3000, False, monkeypatch, dist=dist, dist_param=param)
    for i, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x, y), i


def _switch_seq(gpu, monkeypatch, split):
    import invsim
    monkeypatch.setenv("INVSIM_IM_SPLIT", "1" if split else "0")
    n = 2048
    env = invsim.InvManagementBacklogEnv(n, device=gpu, record_demand=True)
    env.reset(seed=23)
    a = torch.full((n, 3), 15, dtype=torch.int64, device=gpu)
    out = []

    def steps(k):
        for _ in range(k):
            o, r, _, _, info = env.step(a)
            out.extend([o.clone(), r.clone(), info["demand"].clone()])
    steps(3)                                    # numpy, its lookahead cache live
    env.set_demand_stream("philox")
    steps(4)                                    # fast stream, its demand-only cache live
    out.append(env.get_state().clone())         # commit_rng must leave the PCG64 states alone
    steps(2)
    blob = env.get_state().clone()
    steps(3)
    env.set_state(blob)                         # counter from the blob; the cache dropped
    steps(3)
    env.set_demand_stream("numpy")
    steps(4)
    env.reset(seed=5)
    env.set_demand_stream("philox")
    steps(2)
    out.append(env.get_state().clone())
    return out


def test_fast_stream_lookahead_across_switches_and_checkpoints(gpu, monkeypatch):
    """The fast stream's demand-only lookahead (split step kernel) against the
    run kernel over stream switches, get_state / set_state and reseeding: the
    cache is never committed into the PCG64 states and is dropped whenever the
    counter or the key moves."""
    a = _switch_seq(gpu, monkeypatch, True)
    b = _switch_seq(gpu, monkeypatch, False)
    for i, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x.view(torch.uint8) if x.dtype == torch.float64 else x,
                           y.view(torch.uint8) if y.dtype == torch.float64 else y), i


def _net_fast_run(gpu, graph, n, fused, monkeypatch):
    import invsim
    from invsim.topology import custom_graph, default_graph
    for v in ("INVSIM_NET_AHEAD", "INVSIM_NET_ROLL", "INVSIM_NET_POL_ROLL"):
        monkeypatch.setenv(v, "1" if fused else "0")
    monkeypatch.setenv("INVSIM_NET_ROLL3", "0" if n == 40000 else "1")   # 40 000: the 2-role net_roll_kernel
    g = default_graph() if graph == "default" else custom_graph()
    env = invsim.NetInvMgmtBacklogEnv(n, device=gpu, graph=g, demand_stream="philox", record_demand=True)
    env.reset(seed=19)
    gen = torch.Generator(device=gpu)
    gen.manual_seed(6)
    A = env.action_dim
    out = []
    for k in range(33):                                   # split steps with the demand-only lookahead
        a = torch.rand((n, A), device=gpu, generator=gen) * 60
        o, r, te, tr, info = env.step(a)
        out += [o.clone(), r.clone(), tr.clone(), info["demand"].clone()]
    acts = torch.rand((45, n, A), device=gpu, generator=gen) * 60
    out += list(env.rollout(acts))                         # 3-role / 2-role rollout kernels
    m = torch.zeros((n, invsim.policies.metrics_dim(env)), dtype=torch.float64, device=gpu)
    pol = env.rollout_policy(invsim.ConstantOrderAgent(0.1), 40, obs=True, actions=True, metrics=m)
    out += [pol[k] for k in sorted(pol)] + [m]
    out.append(env.get_state())
    return out


@pytest.mark.parametrize("graph,n", [("default", 4096), ("default", 40000), ("custom", 5000)])
def test_fast_stream_net_fused_kernels_equal_spec_kernel(gpu, monkeypatch, graph, n):
    """Net: the fast stream on net_step2_kernel (demand-only lookahead) and the
    rollout kernels (3-role; 2-role for the 40 000-env case) == net_spec_kernel,
    bit for bit."""
    a = _net_fast_run(gpu, graph, n, True, monkeypatch)
    b = _net_fast_run(gpu, graph, n, False, monkeypatch)
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x.view(torch.uint8) if x.dtype == torch.float64 else x,
                           y.view(torch.uint8) if y.dtype == torch.float64 else y), i


def _nv_fast_run(gpu, n, fused, monkeypatch, L=5, limit=40, mu_max=200.0):
    import invsim
    for v in ("INVSIM_NV_AHEAD", "INVSIM_NV_ROLL", "INVSIM_NV_POL_ROLL"):
        monkeypatch.setenv(v, "1" if fused else "0")
    env = invsim.NewsvendorEnv(n, device=gpu, lead_time=L, step_limit=limit, mu_max=mu_max,
                               demand_stream="philox", record_demand=True)
    env.reset(seed=29)
    gen = torch.Generator(device=gpu)
    gen.manual_seed(8)
    out = []
    for k in range(limit + 6):                             # lookahead steps, across the NEXT_STEP reset
        a = torch.rand((n, 1), device=gpu, generator=gen) * 150
        o, r, te, tr, info = env.step(a)
        out += [o.clone(), r.clone(), tr.clone(), info["demand"].clone()]
    acts = torch.rand((2 * limit + 7, n, 1), device=gpu, generator=gen) * 150
    out += list(env.rollout(acts))                         # 3-wave rollout kernel, resets mid-launch
    for ag in (invsim.OrderUpToHeuristicAgent(1.2), invsim.ClassicNewsvendorAgent("profit_margin", 0.9)):
        m = torch.zeros((n, 2), dtype=torch.float64, device=gpu)
        pol = env.rollout_policy(ag, limit + 9, obs=True, actions=True, metrics=m)
        out += [pol[k] for k in sorted(pol)] + [m]
    for k in range(3):                                     # steps after a rollout: a new lookahead chain
        a = torch.rand((n, 1), device=gpu, generator=gen) * 150
        o, r, te, tr, info = env.step(a)
        out += [o.clone(), r.clone(), info["demand"].clone()]
    out.append(env.get_state())
    return out


@pytest.mark.parametrize("n,L,limit,mu_max", [(4096, 5, 40, 200.0), (65536, 5, 40, 200.0),
                                              (5000, 2, 12, 14.0), (3000, 9, 17, 200.0)])
def test_fast_stream_newsvendor_fused_kernels_equal_run_kernel(gpu, monkeypatch, n, L, limit, mu_max):
    """Newsvendor on the fast stream: the lookahead step kernel (demand-only
    cache), the 3-wave rollout kernel (PTRS wave positioned per launch step,
    multiplication draws spread over the wave's lanes) and its in-kernel agents
    give nv_run_kernel's results bit for bit.  mu_max = 14 puts ~70 % of the
    episodes on the multiplication branch (more than the parity kernel's
    16-env lane groups)."""
    a = _nv_fast_run(gpu, n, True, monkeypatch, L, limit, mu_max)
    b = _nv_fast_run(gpu, n, False, monkeypatch, L, limit, mu_max)
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x.view(torch.uint8) if x.dtype == torch.float64 else x,
                           y.view(torch.uint8) if y.dtype == torch.float64 else y), i


def _nv_switch_seq(gpu, monkeypatch, ahead):
    import invsim
    monkeypatch.setenv("INVSIM_NV_AHEAD", "1" if ahead else "0")
    n = 2048
    env = invsim.NewsvendorEnv(n, device=gpu, record_demand=True)
    env.reset(seed=23)
    a = torch.full((n, 1), 40.0, device=gpu)
    out = []

    def steps(k):
        for _ in range(k):
            o, r, _, _, info = env.step(a)
            out.extend([o.clone(), r.clone(), info["demand"].clone()])
    steps(3)                                    # numpy, its lookahead cache live
    env.set_demand_stream("philox")
    steps(4)                                    # fast stream, its demand-only cache live
    out.append(env.get_state().clone())         # the PCG64 states untouched
    steps(2)
    blob = env.get_state().clone()
    steps(3)
    env.set_state(blob)                         # counter from the blob; the cache dropped
    steps(3)
    env.reset()                                 # the reset's own counter value
    steps(2)
    env.set_demand_stream("numpy")
    steps(4)
    env.reset(seed=5)
    env.set_demand_stream("philox")
    steps(2)
    out.append(env.get_state().clone())
    return out


def test_fast_stream_newsvendor_lookahead_across_switches_and_checkpoints(gpu, monkeypatch):
    a = _nv_switch_seq(gpu, monkeypatch, True)
    b = _nv_switch_seq(gpu, monkeypatch, False)
    for i, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x.view(torch.uint8) if x.dtype == torch.float64 else x,
                           y.view(torch.uint8) if y.dtype == torch.float64 else y), i


def test_fast_stream_newsvendor_pit_1e8(gpu):
    """Newsvendor on the fast stream (the lookahead step kernel): each episode
    draws mu ~ U(0, mu_max) and then Poisson(mu) demands, so the randomized
    probability integral transform u = F(d - 1) + V (F(d) - F(d - 1)) with the
    episode's own mu is U(0, 1) whatever mu is.  Over >= 1e8 draws: a
    chi-square on 100 bins of u, separately for numpy's two sampler branches
    (mu < 10: multiplication, mu >= 10: PTRS), and the mean of (d - mu) / sqrt(mu)."""
    import invsim
    from scipy.stats import chi2
    n = 65536
    env = invsim.NewsvendorEnv(n, device=gpu, record_demand=True, demand_stream="philox", copy=False)
    env.reset(seed=13)
    a = torch.zeros((n, 1), device=gpu)
    gen = torch.Generator(device=gpu).manual_seed(17)
    bins = 100
    hist = {b: torch.zeros(bins, dtype=torch.float64, device=gpu) for b in ("mult", "ptrs")}
    zsum = {b: torch.zeros((), dtype=torch.float64, device=gpu) for b in ("mult", "ptrs")}
    cnt = {b: 0 for b in ("mult", "ptrs")}
    mu = env.params()[:, 4].clone()
    draws = 0
    k = 0
    while draws < 100_000_000:
        d = env.step(a)[4]["demand"].double()
        if k % 41 == 40:                                   # the NEXT_STEP reset call: new params, no draw
            mu = env.params()[:, 4].clone()
        else:
            lo = torch.where(d > 0, torch.special.gammaincc(d, mu), torch.zeros_like(d))   # F(d - 1)
            hi = torch.special.gammaincc(d + 1, mu)                                        # F(d)
            u = lo + torch.rand(n, dtype=torch.float64, device=gpu, generator=gen) * (hi - lo)
            z = (d - mu) / mu.clamp(min=1e-300).sqrt()
            for b, m in (("mult", mu < 10), ("ptrs", mu >= 10)):
                ub = u[m]
                hist[b] += torch.bincount((ub * bins).long().clamp(0, bins - 1), minlength=bins).double()
                zsum[b] += z[m].sum()
                cnt[b] += int(m.sum())
            draws += n
        k += 1
    for b in ("mult", "ptrs"):
        h = hist[b].cpu().numpy()
        e = cnt[b] / bins
        stat = float(((h - e) ** 2 / e).sum())
        p = float(chi2.sf(stat, bins - 1))
        assert p > 1e-4, f"{b}: PIT chi-square {stat:.1f} on {bins - 1} dof, p = {p:.2e} ({cnt[b]} draws)"
        assert abs(float(zsum[b]) / cnt[b]) < 6 / np.sqrt(cnt[b]), b
    assert cnt["mult"] > 2_000_000 and cnt["ptrs"] > 90_000_000


@pytest.mark.parametrize("cls", ["InvManagementBacklogEnv", "NewsvendorEnv", "NetInvMgmtBacklogEnv"])
def test_fast_stream_same_seed_replays_demands(gpu, cls):
    """reset(seed=s) twice on one handle gives the same demands on the fast
    stream too: an unmasked seed restarts the launch-step counter.
    Steps, a rollout and a reseed with another seed in between."""
    import invsim
    n = 3000
    env = getattr(invsim, cls)(n, device=gpu, demand_stream="philox", record_demand=True)
    A = env.action_dim
    g = torch.Generator(device=gpu).manual_seed(1)
    acts = [torch.rand((n, A), device=gpu, generator=g) * 40 for _ in range(8)]
    if env.act_dtype != torch.float32:
        acts = [a.to(env.act_dtype) for a in acts]

    def episode(seed):
        obs0, _ = env.reset(seed=seed)
        out = [obs0.clone()]
        for a in acts:
            o, r, _, _, _ = env.step(a)
            out += [o.clone(), r.clone(), env._demand.clone()]
        return out
    first = episode(11)
    env.rollout(torch.stack(acts[:5]))
    episode(12)
    again = episode(11)
    for x, y in zip(first, again):
        assert torch.equal(x, y)
