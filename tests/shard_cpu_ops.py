"""NumPy restatement of :class:`substrafl_amd.sharding.GpuShardOps` for the CPU (gloo) tests of
the client-sharded protocol -- TEST INFRASTRUCTURE: the per-element arithmetic of the reference
(fed_avg.py:221-222: fl(acc + fl(x_k * w_k)) in list order; scaffold.py:262-263,293 in fp64; the
numel == 1 elements through the oracle's NumPy pairwise sum), applied to torch CPU tensor views so
the same ``client_shard_*`` / ``lockstep_*`` code and ``DistTransport`` run over gloo without a
GPU."""

import numpy as np
import torch

from oracle import numpy_pairwise_sum

_NP = {"f32": np.float32, "bf16": np.float32, "f64": np.float64, "f16": np.float16}


def _np(t):
    return t.float().numpy() if t.dtype == torch.bfloat16 else t.numpy()


class CpuShardOps:
    def fedavg_run(self, kind, rows, w, seed, acc):
        n = int(acc.shape[0])
        if n == 0:
            return
        dt = _NP[kind]
        a = np.zeros(n, dt) if seed else _np(acc).astype(dt)
        x = _np(rows)
        for k in range(rows.shape[0]):
            a = (a + (x[k].astype(dt) * dt(w[k])).astype(dt)).astype(dt)
        acc.copy_(torch.from_numpy(a))

    def fedavg_chain(self, kind, rows, w, a, b, seed, out):
        if b > a:
            self.fedavg_run(kind, rows[:, a:b], w, seed, out[a:b])

    def fedavg_products_at(self, kind, rows, w, kbase, K, idx, ws):
        dt = _NP[kind]
        x = _np(rows) if rows.shape[0] else None
        for p, i in enumerate(np.asarray(idx, np.int64)):
            for k in range(rows.shape[0]):
                ws[p, kbase + k] = float(dt(x[k, i].astype(dt) * dt(w[k])))

    def fedavg_products(self, sh, ws):
        self.fedavg_products_at(sh.kind, sh.rows, sh.w, sh.kbase, sh.K, sh.pairwise_idx, ws)

    def fedavg_finish(self, kind, ws, K, pairwise_idx, out):
        wdt = np.float64 if kind == "f64" else np.float32
        odt = _NP[kind]
        for p, i in enumerate(np.asarray(pairwise_idx, np.int64)):
            terms = ws[p, :K].numpy().astype(wdt)
            out[int(i)] = float(odt(wdt(0.0) + numpy_pairwise_sum(terms)))

    def fedavg_combine(self, kind, parts, M, out):
        pk = "f32" if kind == "bf16" else kind
        self.fedavg_chain(pk, parts, np.ones(parts.shape[0]), 0, M, True, out)

    # -- Scaffold ------------------------------------------------------------------------
    def scaffold_run(self, kind, delta, cv, w, seed, finish, c, lr, dacc, cacc):
        n = int(dacc.shape[0])
        if n == 0:
            return
        ad = np.zeros(n) if seed else dacc.numpy().copy()
        ac = np.zeros(n) if seed else cacc.numpy().copy()
        if delta.shape[0]:
            xd, xc = delta.numpy(), cv.numpy()
            for k in range(delta.shape[0]):
                ad = ad + w[k] * xd[k].astype(np.float64)
                ac = ac + w[k] * xc[k].astype(np.float64)
        if finish:
            ac = ac + c[:n].numpy().astype(np.float64)
            ad = lr * ad
        dacc.copy_(torch.from_numpy(ad))
        cacc.copy_(torch.from_numpy(ac))

    def scaffold_chain(self, sh, a, b, seed, finish, dout, cout):
        if b > a:
            self.scaffold_run(sh.kind, sh.delta[:, a:b], sh.cv[:, a:b], sh.w, seed, finish,
                              sh.c[a:b] if finish else None, sh.lr, dout[a:b], cout[a:b])

    def scaffold_products_at(self, kind, delta, cv, w, kbase, K, idx, ws):
        idx = np.asarray(idx, np.int64)
        P = int(idx.size)
        wd = ws[: P * K].view(P, K)
        wc = ws[P * K:].view(P, K + 1)
        xd, xc = delta.numpy(), cv.numpy()
        for p, i in enumerate(idx):
            for k in range(delta.shape[0]):
                wd[p, kbase + k] = float(w[k] * np.float64(xd[k, i]))
                wc[p, kbase + k] = float(w[k] * np.float64(xc[k, i]))

    def scaffold_products(self, sh, ws):
        self.scaffold_products_at(sh.kind, sh.delta, sh.cv, sh.w, sh.kbase, sh.K, sh.pairwise_idx, ws)

    def scaffold_finish(self, sh, ws, dout, cout):
        P = int(sh.pairwise_idx.size)
        wd = ws[: P * sh.K].view(P, sh.K).numpy()
        wc = ws[P * sh.K:].view(P, sh.K + 1).numpy().copy()
        for p, i in enumerate(np.asarray(sh.pairwise_idx, np.int64)):
            wc[p, sh.K] = np.float64(sh.c[int(i)].item())
            dout[int(i)] = float(sh.lr * (0.0 + numpy_pairwise_sum(wd[p])))
            cout[int(i)] = float(0.0 + numpy_pairwise_sum(wc[p]))

    def scaffold_combine(self, sh, dparts, cparts, dout, cout):
        ad, ac = np.zeros(sh.M), np.zeros(sh.M)
        for g in range(dparts.shape[0]):
            ad = ad + 1.0 * dparts[g, : sh.M].numpy()
            ac = ac + 1.0 * cparts[g, : sh.M].numpy()
        ac = ac + sh.c[: sh.M].numpy().astype(np.float64)
        dout[: sh.M] = torch.from_numpy(sh.lr * ad)
        cout[: sh.M] = torch.from_numpy(ac)
