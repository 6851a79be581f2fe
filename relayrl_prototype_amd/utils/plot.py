"""Offline plots of progress.txt runs -- the reference's utils/plot.py API and CLI
(rf/src/native/python/utils/plot.py:17-253): ``get_newest_dataset``, ``get_datasets``,
``get_all_datasets`` (directory prefixes, ``select`` / ``exclude`` substrings, ``legend``),
``plot_data`` (smoothing, a mean / max / min / median estimator over runs with a spread band)
and ``make_plots`` with ``count`` (one curve per run instead of per condition).

seaborn is not installed, so curves are drawn with matplotlib directly; the datasets are pandas
DataFrames with the reference's added columns ``Unit``, ``Condition1``, ``Condition2`` and
``Performance``.

    python -m relayrl_prototype_amd.utils.plot logs/relayrl-reinforce -l base -x Epoch -y AverageEpRet \
        --select s1 --exclude old --count --est max --out curve.png
"""
from __future__ import annotations

import argparse
import json
import os
import os.path as osp
from typing import Dict, List, Optional, Sequence

import numpy as np

DIV_LINE_WIDTH = 50


class _Counters:
    """The reference keeps ``exp_idx`` / ``units`` as module globals; one object per
    ``get_all_datasets`` call here, so two plots in one process number their runs the same."""

    def __init__(self):
        self.exp_idx = 0
        self.units: Dict[str, int] = {}


def _progress_files(logdir: str) -> List[str]:
    out = []
    for root, _, files in os.walk(logdir):
        if "progress.txt" in files:
            out.append(osp.join(root, "progress.txt"))
    return sorted(out)


def get_newest_dataset(data_log_dir: str, return_file_root: bool = False):
    """The newest progress.txt under ``data_log_dir`` as a DataFrame, or its directory with
    ``return_file_root`` (plot.py:90-119); None when there is none."""
    import pandas as pd

    if not osp.exists(data_log_dir):
        return None
    files = _progress_files(data_log_dir)
    if not files:
        return None
    newest = max(files, key=osp.getctime)
    if return_file_root:
        return osp.abspath(osp.dirname(newest))
    return pd.read_table(newest)


def get_datasets(logdir: str, condition: Optional[str] = None, other_algos: bool = False,
                 _ctr: Optional[_Counters] = None) -> list:
    """Every run under ``logdir`` as a DataFrame with ``Unit`` (run index within its condition),
    ``Condition1`` (``condition`` or the run's config exp_name), ``Condition2`` (Condition1 +
    a global run index) and ``Performance`` (AverageTestEpRet if logged, else AverageEpRet)
    (plot.py:122-175).  ``other_algos`` adds the F1 / SJF scheduling baselines the reference's
    schedulers log, as extra conditions."""
    import pandas as pd

    ctr = _ctr or _Counters()
    datasets = []
    for path in _progress_files(logdir):
        root = osp.dirname(path)
        exp_name = None
        try:
            with open(osp.join(root, "config.json")) as f:
                exp_name = json.load(f).get("exp_name")
        except (OSError, ValueError):
            pass
        c1 = condition or exp_name or "exp"
        c2 = f"{c1}-{ctr.exp_idx}"
        ctr.exp_idx += 1
        unit = ctr.units.get(c1, 0)
        ctr.units[c1] = unit + 1
        try:
            data = pd.read_table(path)
        except Exception:  # noqa: BLE001 -- an empty / torn file is skipped like the reference
            print(f"Could not read from {path}")
            continue
        if data.empty:
            continue
        perf = "AverageTestEpRet" if "AverageTestEpRet" in data else "AverageEpRet"
        data["Unit"] = unit
        if other_algos:
            for base in ("F1", "SJF"):
                if base in data:
                    d2 = data.copy()
                    d2["Condition1"] = base
                    d2["Condition2"] = base
                    d2["Performance"] = -data[base]
                    datasets.append(d2)
        data["Condition1"] = c1
        data["Condition2"] = c2
        if perf in data:
            data["Performance"] = data[perf]
        datasets.append(data)
    return datasets


def _expand(all_logdirs: Sequence[str]) -> List[str]:
    """A real directory given with a trailing separator is taken as is; anything else is a
    PREFIX: every entry of its parent directory whose name contains it (plot.py:178-199)."""
    logdirs = []
    for logdir in all_logdirs:
        if osp.isdir(logdir) and logdir.endswith(os.sep):
            logdirs.append(logdir)
            continue
        basedir = osp.dirname(logdir) or "."
        prefix = osp.basename(logdir.rstrip(os.sep))
        if not osp.isdir(basedir):
            continue
        logdirs += sorted(osp.join(basedir, x) for x in os.listdir(basedir) if prefix in x)
    return logdirs


def get_all_datasets(all_logdirs: Sequence[str], legend: Optional[Sequence[str]] = None,
                     select: Optional[Sequence[str]] = None, exclude: Optional[Sequence[str]] = None,
                     other_algos: bool = False, verbose: bool = True) -> list:
    """Expand prefixes, keep logdirs containing every ``select`` substring and none of the
    ``exclude`` ones, then load them -- one legend entry per logdir (plot.py:178-226)."""
    logdirs = _expand(all_logdirs)
    if select:
        logdirs = [d for d in logdirs if all(x in d for x in select)]
    if exclude:
        logdirs = [d for d in logdirs if not any(x in d for x in exclude)]
    if verbose:
        print("Plotting from...\n" + "=" * DIV_LINE_WIDTH + "\n")
        for d in logdirs:
            print(d)
        print("\n" + "=" * DIV_LINE_WIDTH)
    if legend and len(legend) != len(logdirs):
        raise ValueError(f"give one legend title per set of experiments ({len(logdirs)} logdirs, "
                         f"{len(legend)} titles)")
    ctr = _Counters()
    data = []
    for i, d in enumerate(logdirs):
        data += get_datasets(d, legend[i] if legend else None, other_algos, _ctr=ctr)
    return data


def _smooth(y: np.ndarray, k: int) -> np.ndarray:
    """The reference's smoothing: y_s[t] = mean(y[t-k+1 .. t+k-1]) over the valid window."""
    if k <= 1 or len(y) < 2:
        return np.asarray(y, np.float64)
    y = np.asarray(y, np.float64)
    kern = np.ones(k)
    return np.convolve(y, kern, "same") / np.convolve(np.ones_like(y), kern, "same")


def plot_data(data: list, xaxis: str = "Epoch", value: str = "AverageEpRet", condition: str = "Condition1",
              smooth: int = 1, estimator=np.mean, ax=None):
    """One curve per ``condition`` value: ``estimator`` over its runs (aligned on ``xaxis``)
    with a +-1 std band (plot.py:29-87); x axis in scientific notation past 5e3."""
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    ax = ax or plt.gca()
    groups: Dict[str, list] = {}
    for d in data:
        if value in d and xaxis in d and len(d):
            groups.setdefault(str(d[condition].iloc[0]), []).append(d)
    for cond, runs in groups.items():
        n = min(len(r) for r in runs)
        ys = np.stack([_smooth(r[value].to_numpy()[:n], smooth) for r in runs])
        x = runs[0][xaxis].to_numpy()[:n]
        y = estimator(ys, axis=0)
        ax.plot(x, y, label=cond)
        if len(runs) > 1:
            sd = ys.std(0)
            ax.fill_between(x, y - sd, y + sd, alpha=0.2)
    ax.set_xlabel(xaxis)
    ax.set_ylabel(value)
    if groups:
        ax.legend(loc="best", fontsize=8).set_draggable(True)
    xs = [float(np.nanmax(d[xaxis])) for runs in groups.values() for d in runs]
    if xs and max(xs) > 5e3:
        ax.ticklabel_format(style="sci", axis="x", scilimits=(0, 0))
    return sorted(groups)


def make_plots(all_logdirs: Sequence[str], legend=None, xaxis: Optional[str] = None, values=None, count: bool = False,
               font_scale: float = 1.5, smooth: int = 1, select=None, exclude=None, estimator: str = "mean",
               other_algos: bool = False, out: Optional[str] = None):
    """plot.py:229-238: one figure per value; ``count`` draws every run separately
    (Condition2), else one estimator curve per condition (Condition1).  ``out`` saves the
    figures (``{stem}_{value}{ext}`` when there are several) instead of showing them."""
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    data = get_all_datasets(all_logdirs, legend, select, exclude, other_algos, verbose=out is None)
    values = list(values) if isinstance(values, (list, tuple)) else [values or "Performance"]
    cond = "Condition2" if count else "Condition1"
    est = getattr(np, estimator)
    xaxis = xaxis or "Epoch"
    plt.rcParams.update({"font.size": 10 * font_scale / 1.5})
    figs = []
    for v in values:
        fig = plt.figure(figsize=(7, 4))
        plot_data(data, xaxis=xaxis, value=v, condition=cond, smooth=smooth, estimator=est, ax=fig.gca())
        fig.tight_layout(pad=0.5)
        if out:
            base, ext = osp.splitext(out)
            fig.savefig(out if len(values) == 1 else f"{base}_{v}{ext or '.png'}")
        figs.append(fig)
    if not out:
        plt.show()
    return figs


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("logdir", nargs="*")
    ap.add_argument("--legend", "-l", nargs="*")
    ap.add_argument("--xaxis", "-x", default="TotalEnvInteracts")
    ap.add_argument("--value", "-y", default=["Performance"], nargs="*")
    ap.add_argument("--count", action="store_true")
    ap.add_argument("--smooth", "-s", type=int, default=2)
    ap.add_argument("--select", nargs="*")
    ap.add_argument("--exclude", nargs="*")
    ap.add_argument("--est", default="mean")
    ap.add_argument("--other_algos", type=int, default=0)
    ap.add_argument("--out", default="plot.png", help="image path ('' = interactive window)")
    a = ap.parse_args(argv)
    xaxis = a.xaxis
    if xaxis == "TotalEnvInteracts":  # our progress.txt logs EnvSteps / Epoch (utils/logger.py)
        probe = get_all_datasets(a.logdir, a.legend, a.select, a.exclude, bool(a.other_algos), verbose=False)
        if probe and xaxis not in probe[0]:
            xaxis = "EnvSteps" if "EnvSteps" in probe[0] else "Epoch"
    make_plots(a.logdir, a.legend, xaxis, a.value, a.count, smooth=a.smooth, select=a.select, exclude=a.exclude,
               estimator=a.est, other_algos=bool(a.other_algos), out=a.out or None)


if __name__ == "__main__":
    main()
