"""Run the host C++ runtime (libsvm parser, tokenizer, vocab/encoder, shuffles) under
AddressSanitizer + UndefinedBehaviorSanitizer.

Builds build/asan/_runtime*.so with -fsanitize=address,undefined, then re-runs this file in a
child interpreter with libasan/libubsan preloaded (python itself is not instrumented; the
extension is) and drives every entry point with normal, edge-case and malformed inputs.
Exit status 0 = clean.  Usage: python tools/sanitize_runtime.py
"""
import importlib.util
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _exercise(so_path):
    spec = importlib.util.spec_from_file_location("_runtime", so_path)
    rt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rt)
    text = "".join(f"{i % 3} 1:{i * 0.5} 3:{-i} 4:1e-3\n" for i in range(2000)) + "\n# comment\n2 2:7\n"
    labels, indptr, indices, values, maxi = rt.parse_libsvm_buffer(text, 4)
    assert len(labels) == 2001 and maxi == 4 and indptr[-1] == len(indices)
    for bad in ("1 0:3\n", "x 1:2\n", "1 2:3 1:4\n", "1 3:\n", "1 :5\n"):
        try:
            rt.parse_libsvm_buffer(bad, 2)
        except Exception:
            pass
    rt.parse_libsvm_buffer("", 3)
    lines = ["Hello, World! It's a test.", "", "  multiple   spaces\\tand\\nnewlines ", "unicode é ü ß",
             "a" * 5000, "(AP) -- 123.45 'quoted' \"double\""]
    toks = rt.tokenize_batch(lines * 50)
    assert len(toks) == 300
    counts = rt.count_tokens(lines * 50)
    v = rt.Vocab.build(counts, 1, ["<pad>", "<sos>", "<eos>", "<unk>"], True)
    v.set_default_index(3)
    assert v["<pad>"] == 0 and v["never-seen-token"] == 3
    v.lookup_indices(["hello", "zzz"])
    rt.Vocab(["a", "b"])
    enc = v.encode_batch(toks, 1, 2, 16, 0, 0)
    assert enc.shape[0] == 300
    enc = v.encode_batch([[]] * 5, -1, -1, 0, 0, 40)
    p = rt.permutation(100000, 7)
    assert sorted(p.tolist()) == list(range(100000))
    rt.permutation(0, 1)
    print("sanitized runtime: clean")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        _exercise(sys.argv[2])
        return 0
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import build_native
    so = build_native.build_runtime_sanitized(verbose=False)
    libs = [subprocess.run(["gcc", f"-print-file-name={n}"], capture_output=True, text=True).stdout.strip()
            for n in ("libasan.so", "libubsan.so")]
    env = dict(os.environ, LD_PRELOAD=":".join(libs), ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", so], env=env)
    return r.returncode


if __name__ == "__main__":
    sys.exit(main())
