"""Offline plots of progress.txt runs (reference utils/plot.py: get_newest_dataset,
get_datasets, make_plots, CLI).  seaborn is not installed, so this uses matplotlib only.

    python -m relayrl_prototype_amd.utils.plot logs/ --value AverageEpRet --out curve.png
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import os.path as osp
from typing import Dict, List, Optional

import numpy as np

from .logger import read_progress


def get_newest_dataset(logdir: str) -> Optional[str]:
    """Path of the most recently modified progress.txt under ``logdir`` (plot.py:90-119)."""
    files = glob.glob(osp.join(logdir, "**", "progress.txt"), recursive=True)
    return max(files, key=osp.getmtime) if files else None


def get_datasets(logdir: str, condition: Optional[str] = None) -> List[Dict]:
    """Every run under ``logdir`` as {exp_name, condition, path, data} (plot.py:122-170)."""
    out = []
    for path in sorted(glob.glob(osp.join(logdir, "**", "progress.txt"), recursive=True)):
        d = osp.dirname(path)
        exp = osp.basename(d)
        cfg = osp.join(d, "config.json")
        if osp.exists(cfg):
            try:
                exp = json.load(open(cfg)).get("exp_name", exp)
            except ValueError:
                pass
        data = read_progress(path)
        if not data or not next(iter(data.values()), []):
            continue
        out.append({"exp_name": exp, "condition": condition or exp, "path": path, "data": data})
    return out


def smooth(y, k: int):
    if k <= 1 or len(y) < 2:
        return np.asarray(y)
    y = np.asarray(y, dtype=np.float64)
    kern = np.ones(k)
    return np.convolve(y, kern, "same") / np.convolve(np.ones_like(y), kern, "same")


def make_plots(logdirs: List[str], xaxis: str = "Epoch", values=("AverageEpRet",), smooth_k: int = 1,
               out: Optional[str] = None):
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    runs = [r for d in logdirs for r in get_datasets(d)]
    figs = []
    for v in values:
        fig, ax = plt.subplots(figsize=(7, 4))
        groups: Dict[str, List] = {}
        for r in runs:
            if v in r["data"] and xaxis in r["data"]:
                groups.setdefault(r["condition"], []).append(r)
        for cond, rs in groups.items():
            n = min(len(r["data"][v]) for r in rs)
            ys = np.stack([smooth(r["data"][v][:n], smooth_k) for r in rs])
            x = np.asarray(rs[0]["data"][xaxis][:n])
            m = ys.mean(0)
            ax.plot(x, m, label=cond)
            if len(rs) > 1:
                s = ys.std(0)
                ax.fill_between(x, m - s, m + s, alpha=0.2)
        ax.set_xlabel(xaxis)
        ax.set_ylabel(v)
        ax.legend(loc="best", fontsize=8)
        fig.tight_layout()
        if out:
            base, ext = osp.splitext(out)
            fig.savefig(out if len(values) == 1 else f"{base}_{v}{ext or '.png'}")
        figs.append(fig)
    return figs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("logdir", nargs="+")
    ap.add_argument("--xaxis", "-x", default="Epoch")
    ap.add_argument("--value", "-y", nargs="*", default=["AverageEpRet"])
    ap.add_argument("--smooth", "-s", type=int, default=1)
    ap.add_argument("--out", default="plot.png")
    a = ap.parse_args(argv)
    make_plots(a.logdir, a.xaxis, a.value, a.smooth, a.out)


if __name__ == "__main__":
    main()
