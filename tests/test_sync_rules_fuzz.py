"""Property tests of the sync decision rules against the normative spec (SURVEY Appendix A,
from /root/reference/pkg/devspace/sync/evaluater.go:8-192, file_index.go:20-53, tar.go:44-144).

Each rule gets a small executable model written from the spec text; hypothesis drives the
native engine (devspace_amd._native.SyncRules: the same C++ Session code `devspace dev` runs)
with random index states, stats and exclude lists and checks it agrees with the model."""

import io
import os
import tarfile
import tempfile
import time

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

_native = pytest.importorskip("devspace_amd._native")

SEGS = st.sampled_from(["a", "b", "src", "node_modules", ".git", "x.js", "y.py", "logs"])
RELS = st.lists(SEGS, min_size=1, max_size=4).map(lambda p: "/" + "/".join(p))
PATTERNS = st.lists(st.sampled_from(["node_modules/", "*.py", "/src", ".git/", "logs", "b/x.js", "!y.py"]),
                    max_size=3)
MTIMES = st.integers(min_value=1_000_000, max_value=1_000_020)
SIZES = st.integers(min_value=0, max_value=4)
ENTRY = st.fixed_dictionaries({"size": SIZES, "mtime": MTIMES, "is_dir": st.booleans(), "is_symlink": st.booleans(),
                               "local_mtime_ns": st.one_of(st.just(0), MTIMES.map(lambda s: s * 10**9 + 123))})
INDEX = st.dictionaries(RELS, ENTRY, max_size=6)
SETTINGS = settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.too_slow])


def _matches(pats, rel):
    return bool(pats) and _native.gitignore_match(pats, rel)


def _rules(tmp, mode, exclude, dl, ul, index):
    r = _native.SyncRules(tmp, mode, exclude, dl, ul)
    for name, e in index.items():
        r.put(name, **e)
    return r


_TMP = tempfile.mkdtemp(prefix="sync-rules-")


# ---------------------------------------------------------------- models (Appendix A)


def model_should_upload(index, exclude, mode, rel, s, initial):
    if not s["exists"]:
        return False
    if _matches(exclude + ["/.devspace/logs"], rel):  # the sync log is always excluded
        return False
    if s["is_symlink"]:
        return False
    f = index.get(rel)
    if f is not None:
        if s["is_dir"] or f["is_symlink"]:
            return False
        rounded = s["mtime_sec"] + (1 if s["mtime_nsec"] >= 500_000_000 else 0)
        if initial:
            if rounded <= f["mtime"]:
                return False
        elif mode != "compat" and f["local_mtime_ns"]:
            # non-compat refinement: nanosecond mtimes catch two same-size edits in one second
            if s["mtime_sec"] * 10**9 + s["mtime_nsec"] == f["local_mtime_ns"] and s["size"] == f["size"]:
                return False
        elif rounded == f["mtime"] and s["size"] == f["size"]:
            return False
    return True


def model_should_download(index, exclude, dl, name, size, mtime, is_dir, is_symlink):
    if _matches(exclude + ["/.devspace/logs"], name) or _matches(dl, name) or is_symlink:
        return False
    f = index.get(name)
    if f is None:
        return True
    if is_dir:
        return False
    return mtime > f["mtime"] or (mtime == f["mtime"] and size != f["size"])


def model_should_remove_remote(index, exclude, ul, rel):
    if _matches(exclude + ["/.devspace/logs"], rel) or _matches(ul, rel):
        return False
    f = index.get(rel)
    return f is not None and not f["is_symlink"]


# ---------------------------------------------------------------- properties


@SETTINGS
@given(index=INDEX, exclude=PATTERNS, mode=st.sampled_from(["fast", "compat", "helper"]), rel=RELS,
       s=st.fixed_dictionaries({"exists": st.booleans(), "is_dir": st.booleans(), "is_symlink": st.booleans(),
                                "mtime_sec": MTIMES, "mtime_nsec": st.sampled_from([0, 123, 499_999_999, 500_000_000]),
                                "size": SIZES}),
       initial=st.booleans())
def test_should_upload_matches_spec(index, exclude, mode, rel, s, initial):
    r = _rules(_TMP, mode, exclude, [], [], index)
    assert r.should_upload(rel, initial=initial, **s) == model_should_upload(index, exclude, mode, rel, s, initial)


@SETTINGS
@given(index=INDEX, exclude=PATTERNS, dl=PATTERNS, name=RELS, size=SIZES, mtime=MTIMES, is_dir=st.booleans(),
       is_symlink=st.booleans())
def test_should_download_matches_spec(index, exclude, dl, name, size, mtime, is_dir, is_symlink):
    r = _rules(_TMP, "fast", exclude, dl, [], index)
    got = r.should_download(name, size, mtime, is_dir=is_dir, is_symlink=is_symlink)
    assert got == model_should_download(index, exclude, dl, name, size, mtime, is_dir, is_symlink)


@SETTINGS
@given(index=INDEX, exclude=PATTERNS, ul=PATTERNS, rel=RELS)
def test_should_remove_remote_matches_spec(index, exclude, ul, rel):
    r = _rules(_TMP, "fast", exclude, [], ul, index)
    assert r.should_remove_remote(rel) == model_should_remove_remote(index, exclude, ul, rel)


@SETTINGS
@given(index=INDEX, dirs=st.lists(RELS, max_size=4), removed=st.lists(RELS, max_size=3))
def test_index_bookkeeping(index, dirs, removed):
    """CreateDirInFileMap inserts every ancestor as a dir and keeps existing entries;
    RemoveDirInFileMap removes exactly the path and its subtree, only if the path is indexed."""
    r = _rules(_TMP, "fast", [], [], [], index)
    model = {k: dict(v) for k, v in index.items()}
    for d in dirs:
        r.create_dir(d)
        parts = d.split("/")
        for i in range(2, len(parts) + 1):
            model.setdefault("/".join(parts[:i]), {"is_dir": True})
    assert sorted(r.names()) == sorted(model)
    for name in model:
        got = r.get(name)
        assert got is not None and got["is_dir"] == model[name].get("is_dir", False)
    for d in removed:
        r.remove_dir(d)
        if d in model:
            model = {k: v for k, v in model.items() if k != d and not k.startswith(d + "/")}
        assert sorted(r.names()) == sorted(model)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(entries=st.dictionaries(st.sampled_from(["a.txt", "d/b.txt", "d/e/c.txt", "z.bin"]),
                               st.tuples(st.binary(max_size=16), MTIMES, st.one_of(st.none(), MTIMES)), min_size=1),
       data=st.data())
def test_untar_never_overwrites_newer_local_files(entries, data):
    """untarNext: an archive entry is skipped when the local file's mtime is newer; otherwise the
    content and mtime come from the archive and the entry lands in the index."""
    root = tempfile.mkdtemp(prefix="untar-", dir=_TMP)
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        for name, (content, mtime, _) in entries.items():
            ti = tarfile.TarInfo(name)
            ti.size, ti.mtime, ti.mode = len(content), mtime, 0o644
            tf.addfile(ti, io.BytesIO(content))
    for name, (_, _, local_mtime) in entries.items():
        if local_mtime is None:
            continue
        p = os.path.join(root, name)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:
            f.write(b"LOCAL")
        os.utime(p, (local_mtime, local_mtime))
    r = _native.SyncRules(root, "fast", [], [], [])
    r.apply_archive(buf.getvalue())
    for name, (content, mtime, local_mtime) in entries.items():
        p = os.path.join(root, name)
        if local_mtime is not None and local_mtime > mtime:
            assert open(p, "rb").read() == b"LOCAL"
            assert int(os.stat(p).st_mtime) == local_mtime
            assert r.get("/" + name)["mtime"] == local_mtime
        else:
            assert open(p, "rb").read() == content
            assert int(os.stat(p).st_mtime) == mtime
            assert r.get("/" + name) == {"size": len(content), "mtime": mtime, "is_dir": False, "is_symlink": False}
            # every ancestor directory of a written entry is indexed (CreateDirInFileMap); a
            # skipped entry only refreshes its own record, as tar.go does
            parts = ("/" + name).split("/")[:-1]
            for i in range(2, len(parts) + 1):
                assert r.get("/".join(parts[:i]))["is_dir"]


@settings(max_examples=80, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(size=SIZES, mtime=MTIMES, idx_size=SIZES, idx_mtime=MTIMES, local_mtime=MTIMES,
       dl=st.lists(st.sampled_from(["*.txt", "/d", "other"]), max_size=2), tracked=st.booleans())
def test_should_remove_local_matches_spec(size, mtime, idx_size, idx_mtime, local_mtime, dl, tracked):
    root = tempfile.mkdtemp(prefix="rmlocal-", dir=_TMP)
    os.makedirs(os.path.join(root, "d"))
    p = os.path.join(root, "d", "f.txt")
    with open(p, "wb") as f:
        f.write(b"x" * size)
    os.utime(p, (local_mtime, local_mtime))
    r = _native.SyncRules(root, "fast", [], dl, [])
    if tracked:
        r.put("/d/f.txt", size=idx_size, mtime=idx_mtime)
    want = (not _matches(dl, "/d/f.txt") and tracked and mtime == idx_mtime and size == idx_size
            and local_mtime <= mtime)
    assert r.should_remove_local(p, "/d/f.txt", size, mtime) == want
    # kind mismatch (remote says dir, index says file) never removes
    assert not r.should_remove_local(p, "/d/f.txt", size, mtime, is_dir=True)
    # missing local path never removes
    assert not r.should_remove_local(os.path.join(root, "nope"), "/nope", 0, mtime)


def test_models_cover_reference_examples():
    """Spot checks straight from evaluater.go's comments, independent of hypothesis."""
    idx = {"/a.js": {"size": 3, "mtime": 1_000_005, "is_dir": False, "is_symlink": False, "local_mtime_ns": 0}}
    r = _rules(_TMP, "compat", [], [], [], idx)
    same = {"exists": True, "is_dir": False, "is_symlink": False, "mtime_sec": 1_000_005, "mtime_nsec": 0, "size": 3}
    assert not r.should_upload("/a.js", initial=False, **same)
    assert r.should_upload("/a.js", initial=False, **dict(same, size=4))
    assert not r.should_upload("/a.js", initial=True, **same)  # initial: mtime not newer
    assert r.should_download("/a.js", 3, 1_000_006)  # newer remote
    assert r.should_download("/a.js", 4, 1_000_005)  # same mtime, other size
    assert not r.should_download("/a.js", 3, 1_000_004)  # older remote
    assert time.time() > 0
