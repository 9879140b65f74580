#!/usr/bin/env python3
"""Accuracy / localisation-error table: Models A, B (distance + event) and C at the reference schedule.

The reference's claim (README.md:8) is that the multi-level MTL network (A) classifies the event type and
the radial distance better than two single-task networks (B) and the single-level multi-classifier (C),
and is more robust to noise; its trainers score this with sklearn accuracy / confusion matrices
(utils.py:297-322).  With no field data available, this tool trains every model on ONE fixed synthetic
train/validation split (data/synthetic.py, labels balanced over the 16 x 2 classes) at the reference
schedule -- batch 32, 40 epochs, Adam lr 1e-3 / wd 1e-5, LR / 1.5 at every 5th-epoch validation, the
80/20 per-class split -- and evaluates the final model on a held-out test set:

  * ``in-dist``  test samples drawn like the training data (per-sample SNR 6..20 dB);
  * ``snr=S``    clean test signals plus white Gaussian noise at S dB through the reference's
                 ``add_gaussian`` (dataset_preparation.py:83-105; the same fixed noise seed for every model).

Rows: A on the engine (bf16 HIP) and A on plain fp32 PyTorch at the same seed, B_distance, B_event, C, and the
backbone-vs-head ablations A_fc / B_distance_fc (A's / B's backbone with a learned linear head per task in place
of the reference's group-mean head, as Model C's classifier; fp32 PyTorch -- not reference models).

    python tools/accuracy_table.py [--per-class 200] [--epochs 40] [--out gpurun_out/accuracy]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def make_test_sets(per_class: int, seed: int, snrs, device):
    from mtl_das_pytorch_amd.data.mat_dataset import add_gaussian
    from mtl_das_pytorch_amd.data.synthetic import N_DIST, generate
    d = torch.arange(N_DIST).repeat_interleave(2 * per_class)
    e = torch.arange(2).repeat_interleave(per_class).repeat(N_DIST)
    sets = {}
    X, _, _ = generate(len(d), seed=seed, distance=d, event=e)
    sets["in-dist"] = X
    clean, _, _ = generate(len(d), seed=seed + 1, distance=d, event=e, snr_db=(300.0, 300.0))
    c = clean.numpy().astype(np.float64)
    for s in snrs:
        rs = np.random.RandomState(1234 + int(s * 10))
        noisy = np.empty_like(c)
        for i in range(len(c)):  # add_gaussian on each sample's whole matrix, reproducible noise per level
            noisy[i] = add_gaussian(c[i], SNR=s, seed=int(rs.randint(0, 2 ** 31 - 1)))
        sets[f"snr={s:g}dB"] = torch.from_numpy(noisy.astype(np.float32))
    lab2 = torch.stack([d, e], 1)
    joint = d + N_DIST * e
    return {k: v.to(device) for k, v in sets.items()}, lab2.to(device), joint.to(device), e.to(device)


def run_one(name, model, backend, args, seed, test_sets, lab2, joint, ev, out_dir, head="group_mean"):
    from mtl_das_pytorch_amd.engine.trainer import Trainer
    from mtl_das_pytorch_amd.utils.config import TrainConfig
    cfg = TrainConfig(model=model, synthetic=args.per_class, synthetic_seed=args.data_seed, batch_size=32,
                      epoch_num=args.epochs, output_savedir=os.path.join(out_dir, f"{name.replace(' ', '_')}_s{seed}"),
                      backend=backend, seed=seed, save_threshold=2.0, log_every=100, head=head)
    t0 = time.time()
    tr = Trainer(cfg)
    tr.run()
    train_s = time.time() - t0
    lab = joint if model == "multi_classifier" else lab2
    row = {"name": name, "seed": seed, "model": model, "backend": tr.backend_name, "train_s": round(train_s, 1),
           "n_train": tr.n_train, "n_val": tr.n_val, "val": tr.last_val["acc"], "test": {}}
    for k, X in test_sets.items():
        r = tr.evaluate(X, lab)
        row["test"][k] = {"acc": {t: round(v, 4) for t, v in r["acc"].items()},
                          "mae_m": None if r.get("mae_m") is None else round(r["mae_m"], 4)}
        if r.get("distance_cm") is not None:
            row["test"][k]["distance_cm"] = r["distance_cm"]
            row["test"][k]["errors"] = error_profile(np.asarray(r["distance_cm"]))
            # the distance task per event type (is a collapse tied to one event signature?)
            by = []
            for e_ in (0, 1):
                sel = ev == e_
                re_ = tr.evaluate(X[sel], lab[sel])
                cm = np.asarray(re_["distance_cm"])
                by.append({"acc": round(float(np.trace(cm) / cm.sum()), 4), "mae_m": round(re_["mae_m"], 3),
                           "top_pred_class": int(cm.sum(0).argmax()),
                           "top_pred_share": round(float(cm.sum(0).max() / cm.sum()), 3)})
            row["test"][k]["distance_by_event"] = by
    tr.close()  # graphs, captured events and streams of this program released before the next one is built
    print(json.dumps(row), flush=True)
    return row


def error_profile(cm: np.ndarray) -> dict:
    """Where the distance errors go (rows = true class, columns = predicted; 1 m bins): the share of errors
    within one bin of the truth, their mean |error| in metres, the share of all predictions that fall in the
    most-predicted class, and the mean signed error (prediction - truth) -- tells an ordinal near-miss
    localiser from one that collapses noisy samples onto a fixed class."""
    n = cm.sum()
    idx = np.arange(cm.shape[0])
    dist = np.abs(idx[None, :] - idx[:, None])
    err = cm * (dist > 0)
    ne = err.sum()
    top = int(cm.sum(0).argmax())
    return {"near_miss_share": round(float((cm * (dist == 1)).sum() / max(ne, 1)), 4),
            "mean_abs_err_of_errors_m": round(float((err * dist).sum() / max(ne, 1)), 3),
            "top_pred_class": top, "top_pred_share": round(float(cm[:, top].sum() / max(n, 1)), 4),
            "mean_signed_err_m": round(float((cm * (idx[None, :] - idx[:, None])).sum() / max(n, 1)), 3)}


def _stat(vals, fmt):
    vals = [v for v in vals if v is not None]
    if not vals:
        return "—"
    m = float(np.mean(vals))
    return (fmt % m) + (f" ± {fmt % float(np.std(vals))}" if len(vals) > 1 else "")


def to_markdown(rows, args):
    """Mean ± std over seeds: one table for the in-distribution test set, one for the SNR sweep."""
    names = list(dict.fromkeys(r["name"] for r in rows))
    keys = list(rows[0]["test"].keys())
    seeds = sorted({r["seed"] for r in rows})
    lines = [f"Synthetic data: {args.per_class} train+val samples per (distance, event) class "
             f"({32 * args.per_class} total, 80/20 split), {args.test_per_class} test samples per class; "
             f"{args.epochs} epochs, bs 32, Adam 1e-3 / wd 1e-5, LR / 1.5 every 5 epochs; "
             f"mean ± std over seeds {seeds}.", ""]

    def cell(name, key, what):
        rs = [r for r in rows if r["name"] == name]
        if what == "mae":
            return _stat([r["test"][key]["mae_m"] for r in rs], "%.3f")
        return _stat([r["test"][key]["acc"].get(what) for r in rs], "%.4f")

    lines += ["| Model | backend | event acc | distance acc | distance MAE (m) | train s |", "|---|---|---|---|---|---|"]
    for n in names:
        rs = [r for r in rows if r["name"] == n]
        lines.append(f"| {n} | {rs[0]['backend']} | {cell(n, keys[0], 'event')} | {cell(n, keys[0], 'distance')} | "
                     f"{cell(n, keys[0], 'mae')} | {_stat([r['train_s'] for r in rs], '%.0f')} |")
    lines += ["", "Noise robustness (clean test signals + add_gaussian at the given SNR): event acc / distance acc / "
              "distance MAE (m)", "", "| Model | " + " | ".join(keys[1:]) + " |", "|---|" + "---|" * (len(keys) - 1)]
    for n in names:
        lines.append(f"| {n} | " + " | ".join(f"{cell(n, k, 'event')} / {cell(n, k, 'distance')} / {cell(n, k, 'mae')}"
                                           for k in keys[1:]) + " |")
    lines += ["", "Distance errors (error_profile): share of errors within one bin / mean |error| of the errors (m) / "
              "most-predicted class and its share of all predictions / mean signed error (m)", "",
              "| Model | " + " | ".join(keys) + " |", "|---|" + "---|" * len(keys)]
    for n in names:
        rs = [r for r in rows if r["name"] == n]
        if "errors" not in rs[0]["test"][keys[0]]:
            continue

        def prof(k):
            e = [r["test"][k]["errors"] for r in rs]
            tops = sorted({x["top_pred_class"] for x in e})
            return (f"{_stat([x['near_miss_share'] for x in e], '%.2f')} / "
                    f"{_stat([x['mean_abs_err_of_errors_m'] for x in e], '%.1f')} / "
                    f"{','.join(str(t) for t in tops)}: {_stat([x['top_pred_share'] for x in e], '%.2f')} / "
                    f"{_stat([x['mean_signed_err_m'] for x in e], '%+.1f')}")
        lines.append(f"| {n} | " + " | ".join(prof(k) for k in keys) + " |")
    lines += ["", "Distance accuracy per event type (striking / excavating test samples evaluated separately; most-"
              "predicted class and its share)", "", "| Model | " + " | ".join(keys) + " |", "|---|" + "---|" * len(keys)]
    for n in names:
        rs = [r for r in rows if r["name"] == n]
        if "distance_by_event" not in rs[0]["test"][keys[0]]:
            continue

        def byev(k):
            out = []
            for e_ in (0, 1):
                b = [r["test"][k]["distance_by_event"][e_] for r in rs]
                tops = sorted({x["top_pred_class"] for x in b})
                out.append(f"{_stat([x['acc'] for x in b], '%.3f')} ({','.join(map(str, tops))}: "
                           f"{_stat([x['top_pred_share'] for x in b], '%.2f')})")
            return " / ".join(out)
        lines.append(f"| {n} | " + " | ".join(byev(k) for k in keys) + " |")
    return "\n".join(lines) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-class", type=int, default=200)
    ap.add_argument("--test-per-class", type=int, default=50)
    ap.add_argument("--epochs", type=int, default=40)
    ap.add_argument("--seeds", type=str, default="0,1,2", help="init / shuffle seeds (same data split)")
    ap.add_argument("--data-seed", type=int, default=17)
    ap.add_argument("--snr", type=str, default="20,10,5,0,-5")
    ap.add_argument("--rows", type=str, default="A,A_fp32,B_distance,B_event,C")
    ap.add_argument("--out", type=str, default=os.path.join(ROOT, "gpurun_out", "accuracy"))
    ap.add_argument("--runs-dir", type=str, default=None,
                    help="training run directories (resume sidecars are large: default a temp dir)")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    import tempfile
    runs = args.runs_dir or tempfile.mkdtemp(prefix="mda_acc_")
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    snrs = [float(s) for s in args.snr.split(",") if s]
    test_sets, lab2, joint, ev = make_test_sets(args.test_per_class, 99991 + args.data_seed, snrs, dev)
    spec = {"A": ("A MTL_Net", "MTL", "engine"), "A_fp32": ("A MTL_Net (fp32 torch)", "MTL", "torch"),
            "B_distance": ("B Single_Task_Net distance", "single_distance", "engine"),
            "B_event": ("B Single_Task_Net event", "single_event", "engine"),
            "C": ("C Multi_Classifier", "multi_classifier", "engine"),
            "A_fc": ("A backbone + fc head (ablation, fp32 torch)", "MTL", "torch", "fc"),
            "B_distance_fc": ("B distance backbone + fc head (ablation, fp32 torch)", "single_distance", "torch", "fc")}
    rows = []
    for seed in [int(x) for x in args.seeds.split(",")]:
        for key in args.rows.split(","):
            name, model, backend = spec[key][:3]
            head = spec[key][3] if len(spec[key]) > 3 else "group_mean"
            if dev.type != "cuda":
                backend = "torch"
            rows.append(run_one(name, model, backend, args, seed, test_sets, lab2, joint, ev, runs, head=head))
            with open(os.path.join(args.out, "accuracy.json"), "w") as f:
                json.dump({"args": vars(args), "rows": rows}, f, indent=1)
    md = to_markdown(rows, args)
    with open(os.path.join(args.out, "accuracy.md"), "w") as f:
        f.write(md)
    print(md)


if __name__ == "__main__":
    main()
