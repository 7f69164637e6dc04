"""Generate golden vectors from the reference env modules (build container only).

Run from the repo root:

    PYTHONPATH=tests/golden/standin:/root/reference python tests/golden/gen_goldens.py

It imports the reference (`/root/reference/{newsvendor,inventory_management,
network_management,network_management_custom}.py`) through the local gymnasium
stand-in in `tests/golden/standin/` and records, per env instance, every
reset observation and every step's (obs, reward, truncated, info fields).
Nothing from the reference is copied: the fixtures are inputs + outputs only.

Episode protocol recorded for env i (seed = base_seed + i, gymnasium
SyncVectorEnv convention): reset(seed=seed_i); then for each episode
`ep_len` steps; between episodes reset() WITHOUT a seed (RNG stream continues),
exactly what a vector env's autoreset does.

Also records numpy RNG known-answer vectors (SeedSequence -> PCG64 -> random /
poisson), the third-party boundary the reference path calls
(`newsvendor.py:105-111,146`, `inventory_management.py:172`,
`network_management.py:125,263`).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _save(name, cfg, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, config=np.array(json.dumps(cfg)), **arrays)
    print(f"wrote {path} ({os.path.getsize(path)} B)")


# ---------------------------------------------------------------- RNG KATs
def gen_rng():
    seeds = [0, 42, 4000, 123456789, 2**40 + 7, 2**100 + 3]
    lams = [0.3, 5.0, 9.99, 10.0, 20.0, 162.6540478400545]
    n_draw = 1000
    st = np.zeros((len(seeds), 4), dtype=np.uint64)          # state hi, lo, inc hi, lo
    raw = np.zeros((len(seeds), 16), dtype=np.uint64)
    dbl = np.zeros((len(seeds), 16), dtype=np.float64)
    poi = np.zeros((len(seeds), len(lams), n_draw), dtype=np.int64)
    poi_end = np.zeros((len(seeds), len(lams), 2), dtype=np.uint64)  # end state hi/lo
    words = np.zeros((len(seeds), 4), dtype=np.uint32)       # entropy words (<=4)
    nwords = np.zeros(len(seeds), dtype=np.int32)
    for i, s in enumerate(seeds):
        w = []
        x = s
        while True:
            w.append(x & 0xFFFFFFFF)
            x >>= 32
            if x == 0:
                break
        nwords[i] = len(w)
        words[i, : len(w)] = w
        bg = np.random.PCG64(np.random.SeedSequence(s))
        d = bg.state["state"]
        st[i] = [d["state"] >> 64, d["state"] & (2**64 - 1), d["inc"] >> 64, d["inc"] & (2**64 - 1)]
        raw[i] = bg.random_raw(16)
        g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(s)))
        dbl[i] = g.random(16)
        for j, lam in enumerate(lams):
            g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(s)))
            poi[i, j] = [g.poisson(lam) for _ in range(n_draw)]
            e = g.bit_generator.state["state"]["state"]
            poi_end[i, j] = [e >> 64, e & (2**64 - 1)]
    # test.py: seeding.np_random(42) then poisson(lam=20, size=100)
    g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(42)))
    testpy = g.poisson(lam=20, size=100).astype(np.int64)
    _save("rng_kat", {"seeds": [str(s) for s in seeds], "lams": lams},
          entropy_words=words, entropy_nwords=nwords, init_state=st, random_raw=raw,
          random_double=dbl, poisson=poi, poisson_end_state=poi_end, testpy_poisson20=testpy)


# ---------------------------------------------------------------- Newsvendor
def nv_actions(rng, n_env, n_step):
    a = rng.uniform(-100.0, 2600.0, size=(n_env, n_step))
    u = rng.random((n_env, n_step))
    a[u < 0.06] = 0.0
    a[(u >= 0.06) & (u < 0.10)] = 2000.0
    a[(u >= 0.10) & (u < 0.14)] = -5.0
    a[(u >= 0.14) & (u < 0.30)] = np.round(a[(u >= 0.14) & (u < 0.30)] / 7.0)   # small ints
    a[(u >= 0.30) & (u < 0.32)] = np.inf
    a[(u >= 0.32) & (u < 0.33)] = np.nan
    a[(u >= 0.33) & (u < 0.45)] = rng.uniform(0, 60, size=a[(u >= 0.33) & (u < 0.45)].shape)
    return a.astype(np.float32)


def gen_newsvendor(name, kwargs, n_env=16, n_ep=3, base_seed=100, act_seed=7):
    import newsvendor as ref
    env0 = ref.NewsvendorEnv(**kwargs)
    ep_len = env0.step_limit
    O = env0.obs_dim
    S = n_ep * ep_len
    rng = np.random.default_rng(act_seed)
    actions = nv_actions(rng, n_env, S)
    obs = np.zeros((n_env, S, O), np.float32)
    rew = np.zeros((n_env, S), np.float64)
    trunc = np.zeros((n_env, S), np.bool_)
    dem = np.zeros((n_env, S), np.int64)
    reset_obs = np.zeros((n_env, n_ep, O), np.float32)
    params = np.zeros((n_env, n_ep, 5), np.float64)
    for i in range(n_env):
        env = ref.NewsvendorEnv(**kwargs)
        for ep in range(n_ep):
            o, info = env.reset(seed=base_seed + i) if ep == 0 else env.reset()
            reset_obs[i, ep] = o
            params[i, ep] = [env.price, env.cost, env.h, env.k, env.mu]
            for k in range(ep_len):
                s = ep * ep_len + k
                o, r, te, tr, info = env.step(actions[i, s:s + 1])
                obs[i, s], rew[i, s], trunc[i, s], dem[i, s] = o, r, tr, info["demand"]
                assert not te
    cfg = dict(kwargs, n_env=n_env, n_ep=n_ep, ep_len=ep_len, base_seed=base_seed)
    _save(name, cfg, actions=actions, obs=obs, reward=rew, truncated=trunc, demand=dem,
          reset_obs=reset_obs, params=params)


# ---------------------------------------------------------------- InvMgmt
def im_actions(rng, n_env, n_step, c):
    m1 = len(c)
    a = rng.integers(-20, max(c) + 60, size=(n_env, n_step, m1))
    u = rng.random((n_env, n_step))
    a[u < 0.10] = 0
    # adversarial: big orders to stage 2 supplier drive stage-1 inventory negative (off-by-one quirk)
    adv = (u >= 0.10) & (u < 0.25)
    a[adv] = np.array([0] + [c[j] * 3 for j in range(1, m1)])[None, :]
    a[(u >= 0.25) & (u < 0.28)] = 10**12          # huge requests -> huge backlog
    return a.astype(np.int64)


def gen_invmgmt(name, cls_name, kwargs, n_env=16, n_ep=2, base_seed=4000, act_seed=11):
    import inventory_management as ref
    cls = getattr(ref, cls_name)
    env0 = cls(**kwargs)
    ep_len = env0.num_periods
    O = env0.pipeline_length
    m = env0.num_stages
    S = n_ep * ep_len
    rng = np.random.default_rng(act_seed)
    actions = im_actions(rng, n_env, S, list(env0.supply_capacity))
    obs = np.zeros((n_env, S, O), np.int64)
    rew = np.zeros((n_env, S), np.float64)
    trunc = np.zeros((n_env, S), np.bool_)
    dem = np.zeros((n_env, S), np.int64)
    sales = np.zeros((n_env, S, m), np.int64)
    unf = np.zeros((n_env, S, m), np.int64)
    endinv = np.zeros((n_env, S, m - 1), np.int64)
    backlog = np.zeros((n_env, S, m), np.int64)
    reset_obs = np.zeros((n_env, n_ep, O), np.int64)
    for i in range(n_env):
        env = cls(**kwargs)
        for ep in range(n_ep):
            o, info = env.reset(seed=base_seed + i) if ep == 0 else env.reset()
            reset_obs[i, ep] = o
            for k in range(ep_len):
                s = ep * ep_len + k
                o, r, te, tr, info = env.step(actions[i, s])
                obs[i, s], rew[i, s], trunc[i, s] = o, r, tr
                dem[i, s] = info["demand_realized"]
                sales[i, s] = info["sales"]
                unf[i, s] = info["unfulfilled"]
                endinv[i, s] = info["ending_inventory"]
                backlog[i, s] = info["backlog_start_of_next"]
    cfg = dict(kwargs, cls=cls_name, n_env=n_env, n_ep=n_ep, ep_len=ep_len, base_seed=base_seed,
               backlog=bool(env0.backlog))
    _save(name, cfg, actions=actions, obs=obs, reward=rew, truncated=trunc, demand=dem,
          sales=sales, unfulfilled=unf, ending_inventory=endinv, backlog_next=backlog,
          reset_obs=reset_obs)


# ---------------------------------------------------------------- NetInvMgmt
def net_actions(rng, n_env, n_step, A):
    a = rng.uniform(0.0, 400.0, size=(n_env, n_step, A))
    u = rng.random((n_env, n_step, A))
    a[u < 0.15] = np.round(a[u < 0.15]) + 0.5          # exact .5 ties (round half-even)
    a[(u >= 0.15) & (u < 0.22)] = -3.0
    a[(u >= 0.22) & (u < 0.30)] = 0.0
    a[(u >= 0.30) & (u < 0.35)] = rng.uniform(1000, 5000, size=a[(u >= 0.30) & (u < 0.35)].shape)
    return a.astype(np.float32)


def gen_net(name, module, cls_name, kwargs, n_env=8, n_ep=1, base_seed=6000, act_seed=13):
    ref = __import__(module)
    cls = getattr(ref, cls_name)
    env0 = cls(**kwargs)
    ep_len = env0.num_periods
    O = env0.obs_dim
    A = len(env0.reorder_links)
    J = len(env0.main_nodes)
    RL = len(env0.retail_links)
    S = n_ep * ep_len
    rng = np.random.default_rng(act_seed)
    actions = net_actions(rng, n_env, S, A)
    obs = np.zeros((n_env, S, O), np.float32)
    rew = np.zeros((n_env, S), np.float64)
    trunc = np.zeros((n_env, S), np.bool_)
    X = np.zeros((n_env, S, J), np.float64)        # X[t+1]
    U = np.zeros((n_env, S, RL), np.float64)       # U[t+1]
    D = np.zeros((n_env, S, RL), np.float64)       # D[t]
    R = np.zeros((n_env, S, A), np.float64)        # R[t]
    Y = np.zeros((n_env, S, A), np.float64)        # Y[t+1]
    P = np.zeros((n_env, S, J), np.float64)        # per-node profit P[t]
    reset_obs = np.zeros((n_env, n_ep, O), np.float32)
    for i in range(n_env):
        env = cls(**kwargs)
        for ep in range(n_ep):
            o, info = env.reset(seed=base_seed + i) if ep == 0 else env.reset()
            reset_obs[i, ep] = o
            for k in range(ep_len):
                s = ep * ep_len + k
                o, r, te, tr, info = env.step(actions[i, s])
                obs[i, s], rew[i, s], trunc[i, s] = o, r, tr
                X[i, s] = env.X.loc[k + 1].values
                U[i, s] = env.U.loc[k + 1].values
                D[i, s] = env.D.loc[k].values
                R[i, s] = env.R.loc[k].values
                Y[i, s] = env.Y.loc[k + 1].values
                P[i, s] = env.P.loc[k].values
    topo = dict(main_nodes=[int(x) for x in env0.main_nodes],
                reorder_links=[[int(a), int(b)] for a, b in env0.reorder_links],
                retail_links=[[int(a), int(b)] for a, b in env0.retail_links],
                obs_dim=int(O), backlog=bool(env0.backlog))
    cfg = dict(kwargs, module=module, cls=cls_name, n_env=n_env, n_ep=n_ep, ep_len=ep_len,
               base_seed=base_seed, topology=topo)
    _save(name, cfg, actions=actions, obs=obs, reward=rew, truncated=trunc, X=X, U=U, D=D,
          R=R, Y=Y, P=P, reset_obs=reset_obs)


def _tile_rows(rows, n_env, S):
    """Edge actions: row s of `rows` (cycled) for step s, rolled by env index so
    every env sees every edge value at a different period."""
    rows = np.asarray(rows)
    idx = (np.arange(S)[None, :] + np.arange(n_env)[:, None]) % len(rows)
    return rows[idx]


NV_EDGES = [-0.0, 0.0, 1.4e-45, -1.4e-45, 2000.0, 2000.0001, np.nan, np.inf, -np.inf, 3999.5,
            1e38, -1e38, 0.5, 1.5, 4000.0, 123.456]
IM_EDGES = [[2**63 - 1, 0, 0], [0, 2**63 - 1, 2**63 - 1], [-(2**63), 0, -1], [2**62, 2**62, 2**62],
            [2**53 + 1, 0, 0], [0, 0, 0], [1, 1, 1], [100, 200, 230], [101, 201, 231], [-1, -1, -1]]
NET_EDGES = [-0.0, 0.5, 1.5, 2.5, -0.5, 1e30, 3.4e38, -1e30, 1.4e-45, 16777217.0, 7.5, 1e7 + 0.5]


def gen_edges():
    """Adversarial actions at the numeric edges of each env's action handling."""
    import inventory_management as im_ref
    import network_management as net_ref
    import newsvendor as nv_ref
    import warnings
    warnings.simplefilter("ignore")
    for L in (0, 5):
        n, S = 8, 16
        acts = _tile_rows(np.array(NV_EDGES, np.float32), n, S)
        obs = np.zeros((n, S, L + 5), np.float32)
        rew = np.zeros((n, S))
        trunc = np.zeros((n, S), bool)
        dem = np.zeros((n, S), np.int64)
        reset_obs = np.zeros((n, 1, L + 5), np.float32)
        params = np.zeros((n, 1, 5))
        for i in range(n):
            env = nv_ref.NewsvendorEnv(lead_time=L, step_limit=S, mu_max=4.0 if L == 0 else 200.0)
            reset_obs[i, 0], _ = env.reset(seed=900 + i)
            params[i, 0] = [env.price, env.cost, env.h, env.k, env.mu]
            for s in range(S):
                o, r, te, tr, info = env.step(acts[i, s:s + 1])
                obs[i, s], rew[i, s], trunc[i, s], dem[i, s] = o, r, tr, info["demand"]
        cfg = dict(lead_time=L, step_limit=S, mu_max=4.0 if L == 0 else 200.0, n_env=n, n_ep=1,
                   ep_len=S, base_seed=900)
        _save(f"newsvendor_edges_L{L}", cfg, actions=acts[..., None], obs=obs, reward=rew,
              truncated=trunc, demand=dem, reset_obs=reset_obs, params=params)
    n, S = 8, 12
    acts = _tile_rows(np.array(IM_EDGES, np.int64), n, S)
    obs = np.zeros((n, S, 33), np.int64)
    rew = np.zeros((n, S))
    trunc = np.zeros((n, S), bool)
    dem = np.zeros((n, S), np.int64)
    reset_obs = np.zeros((n, 1, 33), np.int64)
    for i in range(n):
        env = im_ref.InvManagementBacklogEnv(periods=S)
        reset_obs[i, 0], _ = env.reset(seed=910 + i)
        for s in range(S):
            o, r, te, tr, info = env.step(acts[i, s])
            obs[i, s], rew[i, s], trunc[i, s], dem[i, s] = o, r, tr, info["demand_realized"]
    _save("invmgmt_edges", dict(cls="InvManagementBacklogEnv", periods=S, n_env=n, n_ep=1, ep_len=S,
                                base_seed=910, backlog=True),
          actions=acts, obs=obs, reward=rew, truncated=trunc, demand=dem, reset_obs=reset_obs)
    n, S = 8, 12
    base = np.array(NET_EDGES, np.float32)
    acts = np.stack([_tile_rows(np.roll(base, j), n, S) for j in range(11)], axis=-1)
    O = 68
    obs = np.zeros((n, S, O), np.float32)
    rew = np.zeros((n, S))
    trunc = np.zeros((n, S), bool)
    D = np.zeros((n, S, 1))
    reset_obs = np.zeros((n, 1, O), np.float32)
    for i in range(n):
        env = net_ref.NetInvMgmtBacklogEnv(num_periods=S)
        reset_obs[i, 0], _ = env.reset(seed=920 + i)
        for s in range(S):
            o, r, te, tr, info = env.step(acts[i, s])
            obs[i, s], rew[i, s], trunc[i, s] = o, r, tr
            D[i, s] = env.D.loc[s].values
    env0 = net_ref.NetInvMgmtBacklogEnv(num_periods=S)
    topo = dict(main_nodes=[int(x) for x in env0.main_nodes],
                reorder_links=[[int(a), int(b)] for a, b in env0.reorder_links],
                retail_links=[[int(a), int(b)] for a, b in env0.retail_links], obs_dim=O, backlog=True)
    _save("net_edges", dict(module="network_management", cls="NetInvMgmtBacklogEnv", num_periods=S,
                            n_env=n, n_ep=1, ep_len=S, base_seed=920, topology=topo),
          actions=acts, obs=obs, reward=rew, truncated=trunc, D=D, reset_obs=reset_obs)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "edges":
        gen_edges()
        return
    assert "/root/reference" in sys.path or any("reference" in p for p in sys.path), \
        "run with PYTHONPATH=tests/golden/standin:/root/reference"
    gen_rng()
    gen_newsvendor("newsvendor_default", {})
    gen_newsvendor("newsvendor_capped_L9", dict(lead_time=9, max_inventory=600, step_limit=25,
                                                mu_max=60.0), act_seed=8, base_seed=300)
    gen_newsvendor("newsvendor_L0", dict(lead_time=0, step_limit=20, mu_max=15.0),
                   act_seed=9, base_seed=500)
    gen_newsvendor("newsvendor_config1", dict(step_limit=30), n_env=1, n_ep=1, base_seed=0)
    gen_invmgmt("invmgmt_backlog_default", "InvManagementBacklogEnv", {})
    gen_invmgmt("invmgmt_lostsales_default", "InvManagementLostSalesEnv", {}, base_seed=5000)
    small = dict(periods=10, I0=[10, 10], p=5, r=[3, 2, 1], k=[1, 1, 1], h=[0.5, 0.2],
                 c=[15, 20], L=[1, 2], dist_param={"mu": 8})
    gen_invmgmt("invmgmt_backlog_small_mu8", "InvManagementBacklogEnv", dict(env_config=small),
                base_seed=42)
    big = dict(periods=12, I0=[30, 40, 50, 60, 70, 80, 90, 100],
               r=[9, 8, 7, 6, 5, 4, 3, 2, 1], k=[0.3, 0.2, 0.1, 0.1, 0.05, 0.05, 0.05, 0.02, 0.01],
               h=[0.2, 0.15, 0.12, 0.1, 0.08, 0.06, 0.04, 0.02], c=[60, 70, 80, 90, 100, 110, 120, 130],
               L=[0, 1, 2, 3, 0, 4, 2, 6], p=11, alpha=0.9, dist_param={"mu": 35})
    gen_invmgmt("invmgmt_lostsales_9stage", "InvManagementLostSalesEnv", big, base_seed=777)
    gen_net("net_backlog_default", "network_management", "NetInvMgmtBacklogEnv", {})
    gen_net("net_lostsales_default", "network_management", "NetInvMgmtLostSalesEnv", {},
            base_seed=6100)
    gen_net("net_master_truelost_alpha", "network_management", "NetInvMgmtMasterEnv",
            dict(backlog=False, alpha=0.95, num_periods=20), base_seed=6200, n_ep=2)
    gen_net("net_custom_backlog", "network_management_custom", "NetInvMgmtLostSalesEnv", {},
            base_seed=6300)


if __name__ == "__main__":
    main()
