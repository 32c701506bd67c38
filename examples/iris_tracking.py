"""BASELINE.json config 1: local in-process run, sklearn iris classifier tracked via the client on CPU.

    python examples/iris_tracking.py --store /tmp/plx/polyaxon.sqlite
"""
import argparse
import time

from sklearn.datasets import load_iris
from sklearn.linear_model import LogisticRegression
from sklearn.model_selection import cross_val_score

from polyaxon_amd.client import Experiment

ap = argparse.ArgumentParser()
ap.add_argument("--store", default="/tmp/plx-iris/polyaxon.sqlite")
ap.add_argument("--C", type=float, default=1.0)
ap.add_argument("--max_iter", type=int, default=200)
a = ap.parse_args()

t0 = time.perf_counter()
with Experiment(project="iris", store_path=a.store) as xp:
    xp.log_params(C=a.C, max_iter=a.max_iter)
    X, y = load_iris(return_X_y=True)
    scores = cross_val_score(LogisticRegression(C=a.C, max_iter=a.max_iter), X, y, cv=5)
    for fold, s in enumerate(scores):
        xp.log_metrics(step=fold, accuracy=float(s))
    xp.log_metrics(accuracy_mean=float(scores.mean()), accuracy_std=float(scores.std()))
print(f"experiment {xp.experiment_id}: accuracy {scores.mean():.4f} ({(time.perf_counter() - t0) * 1e3:.1f} ms "
      f"end-to-end tracked)")
