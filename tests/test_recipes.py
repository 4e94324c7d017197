"""Recipes (one per reference script), trainer loop, checkpoint/resume, metrics and config —
CPU (gloo for the data-parallel cases)."""
import json
import os

import pytest
import torch

from sparkmi.train.config import TrainConfig, parse
from sparkmi.utils.checkpoint import CheckpointManager, load_checkpoint, save_checkpoint
from sparkmi.utils.metrics import MetricsLogger, aggregate, read_jsonl

CPU = ["--device", "cpu", "--no-verbose"]


def test_config_cli_and_env(monkeypatch):
    cfg = parse(TrainConfig, ["--batch-size", "64", "--no-graph", "--lr", "0.5"])
    assert cfg.batch_size == 64 and cfg.graph is False and cfg.lr == 0.5
    monkeypatch.setenv("SPARKMI_WORLD", "4")
    assert parse(TrainConfig, []).world == 4
    assert parse(TrainConfig, ["--world", "2"]).world == 2


def test_metrics_logger(tmp_path):
    p = str(tmp_path / "m.rank0.jsonl")
    m = MetricsLogger(p, every=2)
    for i in range(5):
        m.step(torch.tensor(float(i)), 8)
    m.close()
    recs = read_jsonl(p)
    assert [r["step"] for r in recs] == [2, 4, 5]
    assert recs[0]["loss"] == pytest.approx(0.5) and recs[1]["loss"] == pytest.approx(2.5)
    assert aggregate([p])["samples_per_s"] > 0


def test_mlp_recipe_sequential_learns():
    from sparkmi.recipes import mlp
    r = mlp.main(CPU + ["--epochs", "100", "--lr", "2.0"])
    assert r["steps"] == 100 * 3 and r["n_train"] + r["n_test"] == 150
    assert r["test_acc"] > 85.0
    assert list(r["state_dict"].keys())[0] == "layer_1.weight"


def test_mlp_recipe_data_parallel_gloo():
    from sparkmi.recipes import mlp
    r = mlp.main(CPU + ["--world", "2", "--epochs", "5"])
    assert r["world"] == 2 and r["steps"] == 5 * 2  # 44 rows per shard, batch 30 -> 2 batches


def test_cnn_recipe_small():
    from sparkmi.recipes import cnn
    r = cnn.main(CPU + ["--n-train", "256", "--n-test", "64", "--epochs", "1", "--max-steps", "4"])
    assert r["steps"] == 4 and r["n_test"] == 64 and "state_dict" in r


def test_lstm_recipe_small():
    from sparkmi.recipes import lstm
    r = lstm.main(CPU + ["--n-train", "256", "--n-test", "64", "--max-steps", "3"])
    assert r["steps"] == 3 and r["padding_idx"] >= 4


def test_lstm_recipe_data_parallel_sparse_embedding_gloo():
    """distributed_lstm on 2 executors with the row-sparse embedding-gradient exchange."""
    from sparkmi.recipes import lstm
    r = lstm.main(CPU + ["--world", "2", "--n-train", "256", "--n-test", "64", "--max-steps", "3",
                         "--sparse-embedding"])
    assert r["world"] == 2 and r["steps"] == 3


def test_translator_recipe_small():
    from sparkmi.recipes import translator
    r = translator.main(CPU + ["--n-train", "128", "--max-steps", "2", "--d-model", "64", "--ffn-hidden", "128",
                               "--num-heads", "2", "--max-sequence-length", "32"])
    assert r["steps"] == 2 and r["final_loss"] > 0


def test_translator_recipe_dtype_and_metrics(tmp_path):
    """--dtype: fp32 by default (the reference's precision), bf16 on request, anything else
    refused; the metrics records carry the model TFLOP/s of the step."""
    from sparkmi.recipes import translator
    small = CPU + ["--n-train", "64", "--max-steps", "2", "--d-model", "64", "--ffn-hidden", "128", "--num-heads", "2",
                   "--max-sequence-length", "32", "--log-every", "1"]
    assert translator.parse(translator.TranslatorConfig, small).dtype == "fp32"
    r = translator.main(small + ["--metrics", str(tmp_path / "m")])
    assert r["steps"] == 2 and r["dtype"] == "fp32"
    recs = read_jsonl(str(tmp_path / "m.rank0.jsonl"))
    assert recs and all(rec["tflops"] > 0 for rec in recs)
    rb = translator.main(small + ["--dtype", "bf16"])
    assert rb["steps"] == 2 and rb["dtype"] == "bf16" and rb["final_loss"] > 0
    with pytest.raises(ValueError):
        translator.main(small + ["--dtype", "fp16"])


def test_mllib_recipe(tmp_path):
    from sparkmi.recipes import mllib_mlp
    r = mllib_mlp.run(save_path=str(tmp_path / "model"), verbose=False)
    assert r["test_accuracy"] > 0.8
    assert os.path.exists(tmp_path / "model" / "metadata")


def _tiny_cnn_run(tmp_path, argv):
    from sparkmi.recipes import cnn
    return cnn.main(CPU + ["--n-train", "320", "--n-test", "32", "--ckpt-dir", str(tmp_path / "ck")] + argv)


def test_checkpoint_resume_is_exact(tmp_path):
    full = _tiny_cnn_run(tmp_path / "a", ["--epochs", "2", "--no-resume"])
    part = _tiny_cnn_run(tmp_path / "b", ["--epochs", "2", "--max-steps", "13", "--ckpt-every", "13"])
    assert part["steps"] == 13
    rest = _tiny_cnn_run(tmp_path / "b", ["--epochs", "2"])
    assert rest["resumed_from"].endswith("step_000000013") and rest["steps"] == 20 - 13
    for k, v in full["state_dict"].items():
        torch.testing.assert_close(rest["state_dict"][k], v, rtol=0, atol=0)


def test_checkpoint_atomic_and_retention(tmp_path):
    from sparkmi.models.mlp import MultilayerPerceptron
    from sparkmi.optim import Adam
    from sparkmi.utils.flat import FlatParams
    m = MultilayerPerceptron()
    flat = FlatParams(m, shadow=False)
    opt = Adam(flat, lr=0.1)
    flat.grad.fill_(1.0)
    opt.step()
    mgr = CheckpointManager(str(tmp_path), keep=2)
    for s in (1, 2, 3):
        mgr.save(s, m, opt, epoch=0, cursor=s)
    names = sorted(d for d in os.listdir(tmp_path) if d.startswith("step_"))
    assert names == ["step_000000002", "step_000000003"]
    m2 = MultilayerPerceptron()
    flat2 = FlatParams(m2, shadow=False)
    opt2 = Adam(flat2, lr=0.5)
    meta = mgr.restore(m2, opt2)
    assert meta["cursor"] == 3
    for a, b in zip(m2.parameters(), m.parameters()):
        torch.testing.assert_close(a, b)
    torch.testing.assert_close(opt2.m, opt.m)
    assert opt2.lr == pytest.approx(0.1)
    # overwrite in place keeps a valid checkpoint
    save_checkpoint(str(tmp_path / "x"), m, opt, step=5)
    save_checkpoint(str(tmp_path / "x"), m, opt, step=6)
    assert json.load(open(tmp_path / "x" / "meta.json"))["step"] == 6
    assert not [d for d in os.listdir(tmp_path) if ".tmp-" in d or ".old-" in d]
    assert load_checkpoint(str(tmp_path / "x"))["step"] == 6


def test_trace_ranges_noop_and_enabled():
    from sparkmi.utils import trace
    with trace.range("x"):
        pass
    trace.enable(True)
    try:
        with trace.range("y"):
            trace.mark("z")
    finally:
        trace.enable(False)


def test_pinned_stream_loader_cpu_order():
    """PinnedStreamLoader's CPU path: shuffled epochs cover every row once, in the seeded order."""
    import numpy as np
    from sparkmi.data.dataset import PinnedStreamLoader
    a = np.arange(50 * 3, dtype=np.float32).reshape(50, 3)
    y = np.arange(50)
    loader = PinnedStreamLoader([a, y], 8, "cpu", shuffle=True, seed=2)
    for epoch in range(2):
        order = np.random.default_rng(2 + epoch).permutation(50)
        got = [b[1].numpy() for b in loader]
        assert len(got) == 6
        np.testing.assert_array_equal(np.concatenate(got), order[:48])


def test_multistep_groups_follow_the_metrics_logger():
    """Trainer._group never spans a metrics record: the boundary comes from the logger's own step
    count (restarted at 0 after a resume, log_every clamped to >= 1), so a group's summed loss is
    credited to the interval it belongs to (resume at step % log_every != 0, and
    log_every = 0, both used to mis-credit)."""
    from types import SimpleNamespace

    from sparkmi.train.trainer import Trainer
    from sparkmi.utils.metrics import MetricsLogger

    def sizes(step, log_every, ckpt_every=0, U=16, n=40):
        t = Trainer.__new__(Trainer)
        t.cfg = SimpleNamespace(log_every=log_every, ckpt_every=ckpt_every, max_steps=0)
        t.metrics = MetricsLogger(None, every=log_every)
        t.ckpt = object() if ckpt_every else None
        t.step = step
        it, out = iter(range(n)), []
        while True:
            g = t._group(it, U)
            if not g:
                return out, t.metrics
            out.append(len(g))
            for _ in g:
                t.step += 1
                t.metrics.step(torch.tensor(1.0), 1)

    out, m = sizes(13, 10)  # resumed at 13: the logger flushes every 10 of ITS steps
    assert out[:4] == [10, 10, 10, 10] and all(r["loss"] == 1.0 for r in m.records)
    out, m = sizes(0, 0, n=5)  # log_every 0 -> every step is a record
    assert out == [1] * 5 and [r["loss"] for r in m.records] == [1.0] * 5
    out, _ = sizes(13, 10, ckpt_every=8, n=24)  # checkpoints stay on global-step multiples
    assert out[0] == 3 and all(x <= 8 for x in out)
