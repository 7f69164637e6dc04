"""Single-env views with the reference's per-env API and history attributes.

The reference's benchmark scripts and heuristic agents reach into one env's
internals: ``num_stages, lead_time, dist_param, lt_max, I,
action_log, period`` (BaseStockAgent, benchmark_InvManagementBacklogEnv.py:154-171),
``D, S, U, X, retail_links, main_nodes, num_periods, period`` (evaluate_agent,
benchmark_NetInvMgmtLostSalesEnv.py:264-280), ``lead_time``, the action space
(benchmark_newsvendor.py:104-110), and the step ``info`` dicts.  A view runs one
env on the GPU (a batch of one through the same kernels, with the per-step
record of invsim_set_info_record) and keeps those histories on the host with
the reference's shapes, dtypes and column labels, so such scripts run
unchanged:

    env = invsim.compat.make("InvManagementBacklogEnv", periods=30)
    obs, info = env.reset(seed=0)
    obs, reward, terminated, truncated, info = env.step(np.array([10, 20, 30]))

numpy in and out (the reference's dtypes); reward is a Python float.
Stepping an InvManagement view past ``num_periods`` raises IndexError like the
reference.  NewsvendorEnv's per-step cost components come back with the
NumPy-2 scalar type the reference's expression produces (Python float,
np.float32 or np.float64).
"""
import numpy as np
import torch

from . import _capi


class _View:
    def __init__(self, vec):
        self._v = vec
        self.observation_space = vec.single_observation_space
        self.action_space = vec.single_action_space
        self.np_random = None
        self.period = 0

    def __getattr__(self, name):        # reference attributes (num_stages, lead_time, ...)
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self._v, name)

    @property
    def unwrapped(self):
        return self

    def _act(self, action):
        a = np.asarray(action)
        return torch.as_tensor(a.reshape(1, -1), device=self._v.device)

    def close(self):
        self._v.close()


class InvManagementView(_View):
    def reset(self, *, seed=None, options=None):
        obs, _ = self._v.reset(seed=seed)
        T, m = self._v.num_periods, self._v.num_stages
        self.I = np.zeros((T + 1, m - 1), np.int64)          # inventory_management.py:203-211
        self.T = np.zeros((T + 1, m - 1), np.int64)
        self.R = np.zeros((T, m - 1), np.int64)
        self.D = np.zeros(T, np.int64)
        self.S = np.zeros((T, m), np.int64)
        self.B = np.zeros((T + 1, m), np.int64)
        self.LS = np.zeros((T, m), np.int64)
        self.P = np.zeros(T, np.float32)
        self.action_log = np.zeros((T, m - 1), np.int64)
        self.period = 0
        self.I[0] = self._v.init_inv.astype(np.int64)
        return obs[0].cpu().numpy(), self._info()

    def _info(self):
        return {"period": self.period, "current_inventory_on_hand": self.I[self.period].copy(),
                "current_backlog": self.B[self.period].copy()}

    def step(self, action):
        t, m = self.period, self._v.num_stages
        a = np.asarray(action)
        obs, r, te, tr, info = self._v.step(self._act(a))
        o = obs[0].cpu().numpy()
        s = info["sales"][0].cpu().numpy()
        u = info["unfulfilled"][0].cpu().numpy()
        self.action_log[t] = np.maximum(a, 0).astype(np.int64)
        self.R[t] = s[1:]
        self.D[t] = int(info["demand"][0])
        self.S[t] = s
        if self._v.backlog:
            self.B[t + 1] = u
        else:
            self.LS[t] = u
        reward = float(r[0])
        self.P[t] = reward
        self.I[t + 1] = o[:m - 1]
        self.period = t + 1
        out = self._info()
        out.update({
            "period_profit": np.float64(info["period_profit"][0].item()),
            "revenue": np.float64(info["revenue"][0].item()),
            "procurement_cost": np.float64(info["procurement_cost"][0].item()),
            "holding_cost": np.float64(info["holding_cost"][0].item()),
            "penalty_cost": np.float64(info["penalty_cost"][0].item()),
            "demand_realized": self.D[t], "sales": s, "unfulfilled": u,
            "ending_inventory": self.I[t + 1].copy(), "backlog_start_of_next": self.B[t + 1].copy()})
        return o, reward, bool(te[0]), bool(tr[0]), out


class NetInvMgmtView(_View):
    def reset(self, *, seed=None, options=None):
        import pandas as pd
        obs, _ = self._v.reset(seed=seed)
        v = self._v
        T, J = v.num_periods, len(v.main_nodes)
        mi = lambda links: pd.MultiIndex.from_tuples(links)  # noqa: E731
        # network_management.py:315-326
        self.X = pd.DataFrame(np.zeros([T + 1, J]), columns=v.main_nodes, dtype=np.float64)
        self.Y = pd.DataFrame(np.zeros([T + 1, len(v.reorder_links)]), columns=mi(v.reorder_links), dtype=np.float64)
        self.R = pd.DataFrame(np.zeros([T, len(v.reorder_links)]), columns=mi(v.reorder_links), dtype=np.float64)
        self.S = pd.DataFrame(np.zeros([T, len(v.network_links)]), columns=mi(v.network_links), dtype=np.float64)
        self.D = pd.DataFrame(np.zeros([T, len(v.retail_links)]), columns=mi(v.retail_links), dtype=np.float64)
        self.U = pd.DataFrame(np.zeros([T + 1, len(v.retail_links)]), columns=mi(v.retail_links), dtype=np.float64)
        self.P = pd.DataFrame(np.zeros([T, J]), columns=v.main_nodes, dtype=np.float64)
        self.period = 0
        for j in v.main_nodes:
            self.X.loc[0, j] = v.graph.nodes[j].get("I0", 0)
        return obs[0].cpu().numpy(), self._info()

    def _info(self):
        p = self.period
        info = {"period": p, "inventory": self.X.iloc[p].to_dict(), "pipeline": self.Y.iloc[p].to_dict(),
                "backlog_start": self.U.iloc[p].to_dict()}
        if p > 0:
            info.update({"demand_prev": self.D.iloc[p - 1].to_dict(), "sales_prev": self.S.iloc[p - 1].to_dict(),
                         "profit_node_prev": self.P.iloc[p - 1].to_dict(),
                         "profit_total_prev": self.P.iloc[p - 1].sum()})
        return info

    def step(self, action):
        v, t = self._v, self.period
        obs, r, te, tr, info = v.step(self._act(np.asarray(action, np.float32)))
        g = lambda k: info[k][0].cpu().numpy()  # noqa: E731
        dem = info["demand"][0].cpu().numpy().reshape(-1) if len(v.retail_links) > 1 else \
            np.array([int(info["demand"][0])])
        self.D.iloc[t] = dem.astype(np.float64)
        self.S.loc[t, v.retail_links] = g("sales")
        self.S.loc[t, v.reorder_links] = g("replenishment")
        self.R.iloc[t] = g("replenishment")
        self.U.iloc[t + 1] = g("unfulfilled")
        self.X.iloc[t + 1] = g("inventory")
        self.Y.iloc[t + 1] = g("pipeline")
        self.P.iloc[t] = g("profit")
        total = 0.0
        for pj in g("profit"):
            total += pj
        reward = float(r[0])
        self.period = t + 1
        out = self._info()
        out["profit_period_undiscounted"] = total
        out["profit_period_discounted"] = reward
        return obs[0].cpu().numpy(), reward, bool(te[0]), bool(tr[0]), out


class NewsvendorView(_View):
    def reset(self, *, seed=None, options=None):
        obs, _ = self._v.reset(seed=seed)
        self.period = self.step_count = 0
        return obs[0].cpu().numpy(), self._info()

    def _info(self):
        p = self._v.params()[0].cpu().numpy()
        self.price, self.cost, self.h, self.k, self.mu = (float(x) for x in p)
        # max(1, .) keeps its Python int operand (newsvendor.py:105-106)
        self.price = 1 if self.price == 1.0 else self.price
        self.cost = 1 if self.cost == 1.0 else self.cost
        return {"price": self.price, "cost": self.cost, "holding_cost_rate": self.h, "penalty_cost_rate": self.k,
                "demand_mean": self.mu, "lead_time": self._v.lead_time, "step_count": self.step_count}

    def step(self, action):
        obs, r, te, tr, info = self._v.step(self._act(np.asarray(action, np.float32)))
        self.step_count += 1
        self.period = self.step_count
        out = self._info()
        out["demand"] = int(info["demand"][0])
        typ = (float, np.float32, np.float64, int)
        for k in ("revenue", "purchase_cost", "holding_cost", "lost_sales_penalty"):   # newsvendor.py:195-199
            out[k] = typ[int(info[k + "_kind"][0])](info[k][0].item())
        return obs[0].cpu().numpy(), float(r[0]), bool(te[0]), bool(tr[0]), out


def make(cls_name, device=None, **kwargs):
    """A single-env view of `cls_name` (an invsim env class name) with the
    reference constructor kwargs."""
    import invsim
    cls = getattr(invsim, cls_name)
    fam = cls.family
    vec_kw = dict(num_envs=1, device=device, autoreset_mode="disabled", record_demand=True,
                  record_info=True)
    vec = cls(**vec_kw, **kwargs)
    if fam == _capi.INVSIM_INVMGMT:
        return InvManagementView(vec)
    if fam == _capi.INVSIM_NETINVMGMT:
        return NetInvMgmtView(vec)
    return NewsvendorView(vec)
