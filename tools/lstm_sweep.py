"""Deterministic LSTM recipe runs over a few (lr, epochs) settings (GPU): final loss + test acc."""
import sys

from sparkmi.recipes import lstm

for lr, ep in [tuple(map(float, a.split("x"))) for a in sys.argv[1:]] or [(0.01, 4), (0.02, 4), (0.005, 6)]:
    ep = int(ep)
    r = lstm.main(["--device", "cuda", "--no-verbose", "--n-train", "8000", "--n-test", "800", "--epochs", str(ep),
                   "--lr", str(lr)])
    print(f"lr {lr} epochs {ep}: final_loss {r['final_loss']:.4f} test_acc {r['test_acc']:.1f}", flush=True)
sys.exit(0)
