"""Native build bookkeeping (tools/build_native.py): rebuild decisions follow CONTENT stamps, so a
copied tree whose mtimes look current still rebuilds changed sources, and an unchanged tree
whose mtimes moved does not."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture()
def bn(tmp_path, monkeypatch):
    spec = importlib.util.spec_from_file_location("build_native_t", os.path.join(ROOT, "tools", "build_native.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    monkeypatch.setattr(m, "OBJ", str(tmp_path))
    return m


def test_content_stamp_drives_rebuild(bn, tmp_path):
    src = tmp_path / "k.hip"
    src.write_text("int a;\n")
    obj = tmp_path / "k.o"
    obj.write_text("obj")
    cmd = ["hipcc", "-c", str(src)]
    d = bn._obj_digest(str(src), cmd, "hdr0")
    assert bn._needs(str(obj), d, False)  # no stamp yet
    bn._write_stamp(str(obj), d)
    assert not bn._needs(str(obj), d, False)
    # newer-looking object, changed source: still rebuilt
    src.write_text("int b;\n")
    os.utime(obj, (2e9, 2e9))
    assert bn._needs(str(obj), bn._obj_digest(str(src), cmd, "hdr0"), False)
    # unchanged source but touched: not rebuilt
    src.write_text("int a;\n")
    os.utime(src, (3e9, 3e9))
    assert not bn._needs(str(obj), bn._obj_digest(str(src), cmd, "hdr0"), False)
    # a header or a flag change rebuilds
    assert bn._needs(str(obj), bn._obj_digest(str(src), cmd, "hdr1"), False)
    assert bn._needs(str(obj), bn._obj_digest(str(src), cmd + ["-O0"], "hdr0"), False)
    assert bn._needs(str(obj), d, True)


def test_headers_digest_covers_include_dir(bn):
    assert len(bn._headers_digest()) == 64
