"""The tested binary is provably the tree's: the library
carries a SHA-256 digest of the sources, headers, flags and arch it was
built from (amph_build_id), build() rebuilds whenever the tree's digest
differs from the library's -- by content, not mtimes -- and smoke() /
bench.py recompute the digest from the sources that travelled with the
library and refuse a mismatch."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import build_native as B  # noqa: E402


def test_shipped_library_is_this_trees_build():
    assert B.lib_build_id() == B.tree_digest(), "libamphora_hip.so is stale: run __graft_entry__.build()"


def test_loaded_library_reports_the_same_id():
    import amphora_amd._lib as L
    assert L.build_id() == B.lib_build_id() == L.tree_build_id()
    assert L.check_build_id() == L.build_id()
    assert len(L.build_id()) == 16 and int(L.build_id(), 16) >= 0


def test_digest_covers_content_flags_and_arch(tmp_path):
    d = B.tree_digest()
    assert d == B.tree_digest()  # deterministic
    assert B.tree_digest(flags=["-O2"]) != d
    assert B.tree_digest(arch="gfx942") != d


@pytest.fixture
def fake_tree(tmp_path, monkeypatch):
    """A copy of the real sources and headers under tmp_path, with build()
    pointed at it and hipcc replaced by a stand-in link that writes a file
    carrying the marker and the digest it was asked for."""
    root = tmp_path / "repo"
    deps = []
    for d in B.DEPS:
        dst = root / os.path.relpath(d, ROOT)
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copyfile(d, dst)
        deps.append(str(dst))
    srcs = [str(root / os.path.relpath(s, ROOT)) for s in B.SOURCES]
    lib = str(root / "amphora_amd" / "libamphora_hip.so")
    calls = []

    def fake_compile_link(out, flags, link_flags, objdir, verbose=False, digest=None):
        digest = digest or B.tree_digest(flags=flags)
        calls.append(digest)
        with open(out, "wb") as fh:
            fh.write(b"\x7fELF...." + B.ID_MARK + digest.encode() + b"\0")

    monkeypatch.setattr(B, "ROOT", str(root))
    monkeypatch.setattr(B, "DEPS", deps)
    monkeypatch.setattr(B, "SOURCES", srcs)
    monkeypatch.setattr(B, "LIB", lib)
    monkeypatch.setattr(B, "compile_link", fake_compile_link)
    return root, lib, calls


def test_build_recompiles_after_a_header_edit(fake_tree):
    root, lib, calls = fake_tree
    B.build()
    assert len(calls) == 1 and B.lib_build_id(lib) == B.tree_digest()
    B.build()
    assert len(calls) == 1  # up to date: nothing rebuilt
    hdr = root / "amphora_amd" / "csrc" / "field.hpp"
    before = B.tree_digest()
    st = os.stat(hdr)
    with open(hdr, "a") as fh:
        fh.write("\n// edited\n")
    os.utime(hdr, (st.st_atime, st.st_mtime - 3600))  # an OLDER mtime must not hide the edit
    assert B.tree_digest() != before and not B.up_to_date()
    B.build()
    assert len(calls) == 2 and calls[1] != calls[0]
    assert B.lib_build_id(lib) == B.tree_digest()


def test_same_tree_same_id_anywhere(fake_tree):
    root, lib, calls = fake_tree
    # the copy under tmp_path hashes like the real tree: paths enter relative
    assert B.tree_digest() == B.tree_digest(deps=B.DEPS, root=str(root))
    B.ROOT = ROOT  # (monkeypatch restores it) the real tree, real paths
    assert B.tree_digest(deps=[os.path.join(ROOT, os.path.relpath(d, str(root))) for d in B.DEPS]) == \
        B.tree_digest(deps=B.DEPS, root=str(root))


def test_build_id_unit_compiles(tmp_path):
    """The generated unit builds and exports the id with the marker."""
    import ctypes
    import subprocess
    src = B.write_build_id_source(str(tmp_path), "0123456789abcdef")
    so = str(tmp_path / "id.so")
    subprocess.run(["g++", "-shared", "-fPIC", src, "-o", so], check=True)
    assert B.lib_build_id(so) == "0123456789abcdef"
    f = ctypes.CDLL(so).amph_build_id
    f.restype = ctypes.c_char_p
    assert f() == b"0123456789abcdef"
