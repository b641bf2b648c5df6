"""Two-loop (history) microbenchmark at config 5's parameter count: the HBM-roofline measurement of
SURVEY.md §8(d) ("report it only for cfg 5 and an isolated microbench").

Runs the real solver (lbf_lbfgs_begin / iterate, CPU-reference Wolfe semantics) on the
4096-2048-1024-1 regression MLP (n = 10,489,857 parameters) with a SMALL sample count, so that each
iteration is dominated by the history sweeps rather than the evaluation. After the ring is full
(k = m live pairs), the history kernels of every iteration are timed with HIP events on the library
stream (lbf_prof_*):

  gram_sweep   forms s = x - x_prev, y = g - g_prev into the ring's write slot and streams the k live
               S and k live Y vectors once against (s, y, g)                (reference lbfgs.hpp:77-84,
               120-136: every dot product of the two loops)
  hist_coef    one workgroup: Gram bookkeeping + the two recurrences on 2k+1 coefficients
  combine      p = sum c_i basis_i (fp64 accumulate), x_trial = x + p     (lbfgs.hpp:121-136 axpys)

Algorithmic bytes: B_2loop = (4k + 2) * n * 4 per direction (S and Y read once per
loop, g read, p written). The kernels' own compulsory bytes are also given: gram (2k + 6) n * 4
(k S + k Y + x, x_prev, g, g_prev read, s, y written), combine (2k + 4) n * 4 (k S + k Y + g + x read,
p + x_trial written).

    python bench_two_loop.py [--m 10,20,50] [--samples 4096] [--iters 10]
Prints one JSON line per m.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

HBM_PEAK_GBS = 8000.0


def regression_data(N, In, seed=123):
    """SURVEY.md §8(d) cfg 5 shape: X ~ N(0,1), y = tanh(v.x/64) + 0.01 N(0,1); drawn on the device with
    torch's generator (the reference has no cfg-5 data of its own; only the shape matters here)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.randn(N, In, device="cuda", generator=g)
    v = torch.randn(In, 1, device="cuda", generator=g)
    Y = torch.tanh(X @ v / 64.0) + 0.01 * torch.randn(N, 1, device="cuda", generator=g)
    return X.contiguous(), Y.contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=str, default="10,20,50")
    ap.add_argument("--samples", type=int, default=4096)
    ap.add_argument("--dims", type=str, default="4096,2048,1024,1")
    ap.add_argument("--acts", type=str, default="relu,relu,linear")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    pkg = __graft_entry__.load_package()
    dims = [int(x) for x in a.dims.split(",")]
    acts = a.acts.split(",")
    ctx = pkg.Context(0)
    net = pkg.Mlp(ctx, dims, acts)
    n = net.nparams
    X, Y = regression_data(a.samples, dims[0])
    for m in [int(x) for x in a.m.split(",")]:
        P = net.init_params(123, "cpu")
        run = pkg.LbfgsRun(net, P, X, Y, m=m, max_iters=1 << 30, tol=0.0, record_cap=m + a.iters + 64)
        run.iterate(m + 2)                                  # ring full: k = m live pairs from here on
        torch.cuda.synchronize()
        ctx.prof_select(None)
        ctx.prof_sample(1)
        ctx.prof_enable(True)
        it0 = run.hist.size
        run.iterate(a.iters)
        torch.cuda.synchronize()
        prof = ctx.prof_read()
        ctx.prof_enable(False)
        iters = run.hist.size - it0
        live = run.hist.as_dict()
        run.close()
        out = {"bench": "two_loop", "dims": a.dims, "n": n, "m": m, "samples": a.samples, "iters": iters}
        sec = {}
        for key, (ms, cnt) in prof.items():
            kind = key.split("[")[0]
            if kind in ("gram_sweep", "hist_coef", "combine_sweep"):
                sec[key] = (ms / max(iters, 1) * 1e3, cnt)  # per iteration (a section may launch twice)
        g = [v for k_, v in sec.items() if k_.startswith("gram_sweep")]
        c = [v for k_, v in sec.items() if k_.startswith("combine_sweep")]
        h = [v for k_, v in sec.items() if k_.startswith("hist_coef")]
        if not (g and c and h):
            out["error"] = f"sections missing: {sorted(prof)}"
            print(json.dumps(out), flush=True)
            continue
        acc = live["accepted"]
        k = min(m, int((acc[: it0] == 1).sum()))           # live pairs when the timed sweeps start
        out["k"] = k
        tg, tc, th = g[0][0], c[0][0], h[0][0]
        b_alg = (4 * k + 2) * n * 4
        b_gram = (2 * k + 6) * n * 4
        b_comb = (2 * k + 4) * n * 4
        t_dir = tg + th + tc
        out.update({
            "gram_us": round(tg, 2), "hist_coef_us": round(th, 2), "combine_us": round(tc, 2),
            "direction_us": round(t_dir, 2),
            "gram_GBs": round(b_gram / tg / 1e3, 1), "combine_GBs": round(b_comb / tc / 1e3, 1),
            "roofline": {"bound": "hbm", "achieved": round(b_alg / t_dir / 1e3, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(b_alg / t_dir / 1e3 / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes": b_alg,
                         "note": "(4k+2)*n*4 per direction / (gram + hist_coef + combine) time"},
            "kernel_bytes_frac": round((b_gram + b_comb) / t_dir / 1e3 / HBM_PEAK_GBS, 4),
            "launches": {k_: v[1] for k_, v in sec.items()},
            "last_loss": float(live["loss"][-1]) if len(live["loss"]) else None,
        })
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
