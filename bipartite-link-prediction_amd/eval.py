"""Drop-in for the reference's eval.py: precision@20 and ROC-AUC per method file.

``run_evaluation(examples, methods, precision_at=20)`` (eval.py:10-46) reads
``./data/test/<method>.json`` (eval.py:14) and prints the same two lines per method.
The AUC is sklearn's ``roc_auc_score`` arithmetic (eval.py:26) restated with numpy: the
tie-averaged Mann-Whitney statistic, which is what the trapezoidal ROC area equals; the
precision is eval.py:22-24,31 (stable sort by score, descending, top min(k, n) per user,
summed and divided by len(examples)). It is a consumer of the engine's files, run on the
host; it is not on the accelerated path. ROC curves are drawn only when ``plot=True``.
"""
import numpy as np

import util

COLORS = ["r", "b", "g", "m", "y", "c", "k", "#FF9900", "#006600", "#663300"]


def roc_auc(ys, ps):
    """Area under the ROC curve of labels ys (0/1) and scores ps, ties averaged."""
    ys = np.asarray(ys, dtype=np.float64)
    ps = np.asarray(ps, dtype=np.float64)
    n = len(ys)
    npos = ys.sum()
    nneg = n - npos
    if npos == 0 or nneg == 0:
        raise ValueError("Only one class present in y_true. ROC AUC score is not defined in that case.")
    order = np.argsort(ps, kind="mergesort")
    sp = ps[order]
    # average rank of each tie group (1-based)
    starts = np.r_[0, np.flatnonzero(np.diff(sp)) + 1]
    ends = np.r_[starts[1:], n]
    avg = 0.5 * (starts + ends - 1) + 1.0
    ranks = np.empty(n, np.float64)
    ranks[order] = np.repeat(avg, ends - starts)
    return float((ranks[ys == 1].sum() - npos * (npos + 1) / 2.0) / (npos * nneg))


def precision_at_k(examples, predictions, k=20):
    total = 0.0
    for u in predictions:
        pairs = [(examples[u][b], predictions[u][b]) for b in predictions[u]]
        n = min(k, len(pairs))
        top = sorted(pairs, key=lambda t: t[1], reverse=True)[:n]
        total += sum(t[0] for t in top) / float(n)
    return total / len(examples)


def grouped_precision_at_k(labels, scores, group_start, n_examples, k=20):
    """Vectorised eval.py:22-24,31 over flat arrays; pairs of one user are contiguous,
    group_start holds each user's first index (ties keep file order: stable sort)."""
    labels = np.asarray(labels)
    scores = np.asarray(scores, dtype=np.float64)
    gid = np.repeat(np.arange(len(group_start)), np.diff(np.r_[group_start, len(labels)]))
    order = np.lexsort((np.arange(len(scores)), -scores, gid))
    pos_in_group = np.arange(len(order)) - np.asarray(group_start)[gid[order]]
    size = np.diff(np.r_[group_start, len(labels)])
    nk = np.minimum(k, size)
    take = pos_in_group < nk[gid[order]]
    hits = np.bincount(gid[order][take], weights=labels[order][take].astype(np.float64), minlength=len(size))
    return float((hits / np.maximum(nk, 1)).sum() / n_examples)


def run_evaluation(examples, methods, precision_at=20, data_dir="./data/test/", plot=False):
    curve_args = []
    results = {}
    for i, method in enumerate(methods):
        predictions = util.load_scores(data_dir + method + ".json")  # the .npz sidecar when present (util.write_sidecar)
        all_ys, all_ps = [], []
        for u in predictions:
            for b in predictions[u]:
                all_ys.append(examples[u][b])
                all_ps.append(predictions[u][b])
        p_at = precision_at_k(examples, predictions, precision_at)
        auc = roc_auc(all_ys, all_ps)
        results[method] = {"precision": p_at, "auc": auc}
        curve_args.append((all_ys, all_ps, method, COLORS[i % len(COLORS)]))
        print("Method:", method)
        print("  Precision @{:} = {:.4f}".format(precision_at, p_at))
        print("  ROC Auc = {:.4f}".format(auc))
    if plot and len(methods) <= len(COLORS):
        import matplotlib.pyplot as plt
        from sklearn.metrics import roc_curve

        plt.figure(figsize=(9, 9))
        plt.xlabel("False Positive Rate")
        plt.ylabel("True Positive Rate")
        plt.xlim([0.0, 1.0])
        plt.title("ROC curves")
        for ys, ps, label, color in curve_args:
            fpr, tpr, _ = roc_curve(ys, ps)
            plt.plot(fpr, tpr, label=label, color=color)
        plt.legend(loc="best")
        plt.show()
    return results


if __name__ == "__main__":
    run_evaluation(util.load_json("data/test/examples.json"),
                   ["examples", "u_adamic", "u_cn", "u_jaccard", "b_adamic", "b_cn", "b_jaccard",
                    "random_baseline", "svd", "random_walks", "weighted_random_walks",
                    "supervised_random_walks", "supervised_classifier"])
