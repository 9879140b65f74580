"""Training-curve PNGs and confusion-matrix SVGs (reference utils.py:51-75, 180-221).

The reference draws the heat-map with seaborn; seaborn is not a dependency here, so the same figure
(annotated integer cells, "OrRd" colour map, bold tick labels, "Predicted Value" / "True Value"
axes) is drawn with matplotlib alone.
"""
from __future__ import annotations

import glob
import os
from typing import Sequence

import numpy as np


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def draw_confusion_matrix(confusion_matrix: np.ndarray, leibie1: Sequence[str], font_scale=2.5, y_offset=0.5,
                          title1=" ", is_show=False, is_save=True, savepath="./cm.svg", figsize=(7, 6.8)):
    plt = _plt()
    cm = np.asarray(confusion_matrix)
    fig, ax = plt.subplots(figsize=figsize)
    ax.imshow(cm, cmap="OrRd", aspect="auto")
    vmax = cm.max() if cm.size else 0
    for i in range(cm.shape[0]):
        for j in range(cm.shape[1]):
            ax.text(j, i, f"{int(cm[i, j])}", ha="center", va="center", fontsize=16 if cm.shape[0] <= 4 else 8,
                    fontweight="bold", color="white" if vmax and cm[i, j] > 0.6 * vmax else "black")
    ax.set_xticks(np.arange(len(leibie1)))
    ax.set_yticks(np.arange(len(leibie1)))
    ax.set_xticklabels(leibie1, fontsize=16 if len(leibie1) <= 4 else 9, fontweight="bold")
    ax.set_yticklabels(leibie1, fontsize=16 if len(leibie1) <= 4 else 9, fontweight="bold")
    ax.set_xlabel("Predicted Value", fontsize=16, fontweight="bold")
    ax.set_ylabel("True Value", fontsize=16, fontweight="bold")
    ax.set_title(title1)
    fig.tight_layout()
    if is_save:
        fig.savefig(savepath)
    if is_show:
        plt.show()
    plt.close(fig)


LINE_NAMES = ("trainAccLine", "trainLossLine", "testAccLine", "testLossLine")


def plot_curves(save_dir: str, model_type: str):
    """Re-load the four curve .npy files and plot them (reference utils.py:180-204).  Missing or empty
    curves are plotted as empty axes instead of crashing (the reference crashes when an epoch has fewer
    than 100 batches)."""
    plt = _plt()
    for name in LINE_NAMES:
        path = os.path.join(save_dir, name + ".npy")
        line = np.load(path, allow_pickle=False) if os.path.exists(path) else np.zeros((2, 0))
        line = np.atleast_2d(line)
        fig = plt.figure()
        if model_type == "MTL":
            labels = ["distance", "event"]
        elif model_type in ("single_distance", "single_event"):
            labels = [model_type]
        elif name in ("trainLossLine", "testLossLine"):
            labels = [model_type]
        else:
            labels = ["distance", "event"]
        for i, lab in enumerate(labels):
            if i < line.shape[0]:
                plt.plot(line[i], label=lab)
        plt.legend()
        fig.savefig(os.path.join(save_dir, name + ".png"))
        plt.close(fig)


def plot_confusion_files(save_dir: str):
    """Test mode: draw every saved ``confusion matrix*.npy`` as an SVG (reference utils.py:207-221)."""
    event_labels = ["Striking", "Excavating "]
    dist_labels = ["{}m".format(i) for i in range(16)]
    for path in sorted(glob.glob(os.path.join(save_dir, "confusion matrix*.npy"))):
        mat = np.load(path, allow_pickle=False)
        if mat.shape[-1] == 16:
            draw_confusion_matrix(mat, dist_labels, figsize=(6.5, 6),
                                  savepath=os.path.join(save_dir, "confusion matrix distance.svg"))
        elif mat.shape[-1] == 2:
            draw_confusion_matrix(mat, event_labels, figsize=(4.5, 4),
                                  savepath=os.path.join(save_dir, "confusion matrix event.svg"))
