"""Recipes end-to-end on one MI355X (HIP graph step capture, fused kernels, HBM loaders)."""
import pytest
import torch

GPU = ["--device", "cuda", "--no-verbose"]


@pytest.mark.gpu
def test_cnn_recipe_gpu_learns():
    from sparkmi.recipes import cnn
    r = cnn.main(GPU + ["--n-train", "6400", "--n-test", "1000", "--epochs", "2", "--lr", "0.1"])
    assert r["steps"] == 400 and r["test_acc"] > 90.0


@pytest.mark.gpu
def test_cnn_recipe_gpu_bf16_learns():
    from sparkmi.recipes import cnn
    r = cnn.main(GPU + ["--n-train", "6400", "--n-test", "1000", "--epochs", "2", "--lr", "0.1", "--conv-dtype", "bf16"])
    assert r["steps"] == 400 and r["test_acc"] > 90.0


@pytest.mark.gpu
def test_cnn_recipe_gpu_resume_exact(tmp_path):
    from sparkmi.recipes import cnn
    base = GPU + ["--n-train", "640", "--n-test", "64", "--epochs", "2"]
    full = cnn.main(base + ["--ckpt-dir", str(tmp_path / "a"), "--no-resume"])
    full2 = cnn.main(base + ["--ckpt-dir", str(tmp_path / "a2"), "--no-resume"])
    cnn.main(base + ["--ckpt-dir", str(tmp_path / "b"), "--max-steps", "25", "--ckpt-every", "25"])
    rest = cnn.main(base + ["--ckpt-dir", str(tmp_path / "b")])
    assert rest["steps"] == 40 - 25
    # no float atomics anywhere in the CNN step (per-image slabs, fixed-order reductions): two
    # uninterrupted runs are bit-identical, and so is a run resumed from a checkpoint
    for k, v in full["state_dict"].items():
        assert torch.equal(full2["state_dict"][k], v), k
        assert torch.equal(rest["state_dict"][k], v), k


@pytest.mark.gpu
def test_lstm_recipe_gpu_deterministic_and_learns():
    """The LSTM step has no float atomics (slab + fixed-order reductions, position-ordered
    embedding backward), so two identical runs are bit-identical; and training beats chance
    (4 classes) by a wide margin."""
    from sparkmi.recipes import lstm
    # deterministic trajectories (tools/lstm_sweep.py): this small LSTM's loss plateau makes some
    # (lr, epochs) settings succeed or stall depending on the (fixed) summation order of a given
    # build; lr 0.03 x 4 epochs reached 99.7 / 98.0 / 99.1 % across three reduction orders
    args = GPU + ["--n-train", "8000", "--n-test", "800", "--epochs", "4", "--lr", "0.03"]
    r1 = lstm.main(args)
    r2 = lstm.main(args)
    assert r1["final_loss"] == r2["final_loss"] and r1["test_acc"] == r2["test_acc"]
    assert r1["test_acc"] > 90.0


@pytest.mark.gpu
def test_translator_recipe_gpu():
    from sparkmi.recipes import translator
    r = translator.main(GPU + ["--n-train", "640", "--max-steps", "15", "--d-model", "128", "--ffn-hidden", "256",
                               "--num-heads", "2", "--max-sequence-length", "64"])
    assert r["steps"] == 15 and r["final_loss"] < 6.0


@pytest.mark.gpu
def test_mlp_recipe_gpu():
    from sparkmi.recipes import mlp
    r = mlp.main(GPU + ["--epochs", "100", "--lr", "2.0"])
    assert r["test_acc"] > 85.0


def _phase_recs(path):
    from sparkmi.utils.metrics import read_jsonl
    recs = read_jsonl(path)
    return [r for r in recs if "fwd_bwd_s" in r]


@pytest.mark.gpu
def test_translator_graph_metrics_phases(tmp_path):
    """A HIP-graph training run (fp32 default) writes metrics records with the per-phase device
    times (fwd_bwd_s / allreduce_s / optim_s from events between the phase graphs) and TFLOP/s."""
    from sparkmi.recipes import translator
    r = translator.main(GPU + ["--n-train", "640", "--max-steps", "12", "--d-model", "128", "--ffn-hidden", "256",
                               "--num-heads", "2", "--max-sequence-length", "64", "--log-every", "4",
                               "--phase-timing", "--metrics", str(tmp_path / "m")])
    assert r["steps"] == 12 and r["dtype"] == "fp32"
    recs = _phase_recs(str(tmp_path / "m.rank0.jsonl"))
    assert recs, "no phase record"
    last = recs[-1]
    assert last["fwd_bwd_s"] > 0 and last["optim_s"] > 0 and last["allreduce_s"] >= 0 and last["tflops"] > 0, last


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_translator_graph_dp_metrics_phases(tmp_path, monkeypatch):
    """The same from a 2-executor data-parallel graph run (split-graph backward, gloo on the
    shared GPU): the allreduce phase is what finish() still waits for after the replays."""
    from sparkmi.recipes import translator
    monkeypatch.setenv("SPARKMI_DIST_BACKEND", "gloo")  # RCCL needs one device per rank
    monkeypatch.setenv("SPARKMI_SHARE_GPUS", "1")       # both executors on the box's one GPU
    monkeypatch.setenv("SPARKMI_DP_COMM", "rccl")      # the process-group path, not the IPC kernel
    r = translator.main(GPU + ["--world", "2", "--n-train", "640", "--epochs", "3", "--max-steps", "12", "--d-model", "128",
                               "--ffn-hidden", "256", "--num-heads", "2", "--max-sequence-length", "64",
                               "--log-every", "4", "--phase-timing", "--metrics", str(tmp_path / "m")])
    assert r["steps"] == 12 and r["world"] == 2
    recs = _phase_recs(str(tmp_path / "m.rank0.jsonl"))
    assert recs and recs[-1]["fwd_bwd_s"] > 0 and recs[-1]["allreduce_s"] >= 0 and recs[-1]["optim_s"] > 0, recs
