"""NumPy restatement of :class:`substrafl_amd.sharding.GpuShardOps` for the CPU (gloo) tests of
the client-sharded protocol -- TEST INFRASTRUCTURE: the per-element arithmetic of the reference
(fed_avg.py:221-222: fl(acc + fl(x_k * w_k)) in list order; scaffold.py:262-263,293 in fp64; the
numel == 1 elements through the oracle's NumPy pairwise sum), applied to torch CPU tensors so the
same ``client_shard_*`` code and ``DistTransport`` run over gloo without a GPU."""

import numpy as np
import torch

from oracle import numpy_pairwise_sum

_NP = {"f32": np.float32, "bf16": np.float32, "f64": np.float64, "f16": np.float16}


def _np(t):
    return t.float().numpy() if t.dtype == torch.bfloat16 else t.numpy()


class CpuShardOps:
    def fedavg_chain(self, kind, rows, w, a, b, seed, out):
        if b <= a:
            return
        dt = _NP[kind]
        acc = np.zeros(b - a, dt) if seed else _np(out[a:b]).astype(dt)
        x = _np(rows)
        for k in range(rows.shape[0]):
            acc = (acc + (x[k, a:b].astype(dt) * dt(w[k])).astype(dt)).astype(dt)
        out[a:b] = torch.from_numpy(acc)

    def fedavg_products(self, sh, ws):
        dt = _NP[sh.kind]
        x = _np(sh.rows) if sh.Kr else None
        for p, i in enumerate(np.asarray(sh.pairwise_idx, np.int64)):
            for k in range(sh.Kr):
                prod = dt(x[k, i].astype(dt) * dt(sh.w[k]))
                ws[p, sh.kbase + k] = float(prod)

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
    def scaffold_chain(self, sh, a, b, seed, finish, dout, cout):
        if b <= a:
            return
        ad = np.zeros(b - a) if seed else dout[a:b].numpy().copy()
        ac = np.zeros(b - a) if seed else cout[a:b].numpy().copy()
        if sh.Kr:
            xd, xc = sh.delta.numpy(), sh.cv.numpy()
            for k in range(sh.Kr):
                ad = ad + sh.w[k] * xd[k, a:b].astype(np.float64)
                ac = ac + sh.w[k] * xc[k, a:b].astype(np.float64)
        if finish:
            ac = ac + sh.c[a:b].numpy().astype(np.float64)
            ad = sh.lr * ad
        dout[a:b] = torch.from_numpy(ad)
        cout[a:b] = torch.from_numpy(ac)

    def scaffold_products(self, sh, ws):
        P = int(sh.pairwise_idx.size)
        wd = ws[: P * sh.K].view(P, sh.K)
        wc = ws[P * sh.K:].view(P, sh.K + 1)
        xd, xc = sh.delta.numpy(), sh.cv.numpy()
        for p, i in enumerate(np.asarray(sh.pairwise_idx, np.int64)):
            for k in range(sh.Kr):
                wd[p, sh.kbase + k] = float(sh.w[k] * np.float64(xd[k, i]))
                wc[p, sh.kbase + k] = float(sh.w[k] * np.float64(xc[k, i]))

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
