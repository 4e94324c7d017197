"""LSTM recipe run-to-run variance / learning-rate check on one GPU:
RUNS runs per setting of (lr, epochs); prints test accuracy and final loss per run."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkmi.recipes import lstm  # noqa: E402

base = ["--device", "cuda", "--no-verbose", "--n-train", "8000", "--n-test", "800"]
settings = [s.split(":") for s in os.environ.get("SETTINGS", "0.01:2").split(",")]
for lr, ep in settings:
    for i in range(int(os.environ.get("RUNS", "3"))):
        r = lstm.main(base + ["--epochs", ep, "--lr", lr])
        print(f"lr {lr} epochs {ep} run {i} acc {r['test_acc']:.2f} loss {r.get('final_loss')}", flush=True)
