"""GPU images keep their slow layer across edits.

The rocm-pytorch Dockerfiles (the example's and the one `devspace init` writes) copy the workload
kit, compile the fused gfx950 ops (~2 min of hipcc) and only then copy the project. The local
dockerd computes the classic builder's per-instruction cache keys (instruction text chained with
the previous key, plus the content of what a COPY copies), so the test sees which layers a
rebuild after an edit of train.py reuses without executing RUN: the kernel-build layer keeps its
key and is "Using cache"; only the last COPY is new. The reference's counterpart is rebuilding
only what changed (/root/reference/pkg/devspace/image/build.go:189-238).
"""
import os

from conftest import DevspaceEnv


def _cluster(tmp_path, gpus=1):
    from devspace_amd.localkube import LocalCluster

    c = LocalCluster(str(tmp_path / "state"), gpus=gpus).start()
    return c, DevspaceEnv(c, str(tmp_path))


def _wait_false(proj):
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    raw = open(cfg_path).read()
    if "wait: false" not in raw:
        raw = raw.replace("chartPath: ./chart", "chartPath: ./chart\n    wait: false")
    open(cfg_path, "w").write(raw)


def _image_history(cluster, ns):
    dep = cluster.store.list("apps", "deployments", ns)[0]
    ref = dep["spec"]["template"]["spec"]["containers"][0]["image"]
    img = cluster.images.resolve(ref)
    assert img, ref
    return ref, img["config"]["History"], img["config"]["RootFS"]["Layers"]


def _check_rebuild_reuses_the_kernel_layer(cluster, lk, proj, ns):
    _wait_false(proj)
    lk.run(["deploy"], proj, timeout=180)
    ref1, h1, layers1 = _image_history(cluster, ns)
    with open(os.path.join(proj, "train.py"), "a") as f:
        f.write("\n# an edit\n")
    out = lk.run(["deploy"], proj, timeout=180).stdout
    ref2, h2, layers2 = _image_history(cluster, ns)
    assert ref1 != ref2, out  # rebuilt: the context changed
    steps1 = [h["created_by"] for h in h1]
    steps2 = [h["created_by"] for h in h2]
    assert steps1 == steps2
    run = next(i for i, s in enumerate(steps2) if s.startswith("RUN python -m devspace_amd.ops.build"))
    kit = next(i for i, s in enumerate(steps2) if s.startswith("COPY devspace_amd/"))
    last_copy = max(i for i, s in enumerate(steps2) if s.startswith("COPY"))
    assert kit < run < last_copy, steps2
    # everything up to and including the kernel build is the same layer, taken from the cache
    for i in range(last_copy):
        assert h1[i]["key"] == h2[i]["key"], (i, steps2[i])
        assert h2[i]["cached"], (i, steps2[i])
    assert h1[last_copy]["key"] != h2[last_copy]["key"] and not h2[last_copy]["cached"]
    # exactly one filesystem layer differs: the project copy
    assert len(layers1) == len(layers2)
    assert [a == b for a, b in zip(layers1, layers2)].count(False) == 1, (layers1, layers2)


def test_example_rebuild_after_an_edit_reuses_the_kernel_build(tmp_path):
    cluster, lk = _cluster(tmp_path)
    try:
        proj = lk.project("rocm-pytorch")
        _check_rebuild_reuses_the_kernel_layer(cluster, lk, proj, "rocm-pytorch")
    finally:
        cluster.stop()


def test_init_generated_dockerfile_rebuild_reuses_the_kernel_build(tmp_path):
    cluster, lk = _cluster(tmp_path)
    try:
        proj = os.path.join(lk.base, "init-layers")
        os.makedirs(proj)
        with open(os.path.join(proj, "train.py"), "w") as f:
            f.write("import torch\nprint(torch.__version__)\n")
        answers = "\n1\nlayers-ns\n\nlocal.registry\nlocal.registry/layers\nno\n"
        lk.run(["init"], proj, input=answers)
        df = open(os.path.join(proj, "Dockerfile")).read()
        assert df.index("COPY devspace_amd/ devspace_amd/") < df.index("RUN python -m devspace_amd.ops.build") \
            < df.index("COPY . .")
        _check_rebuild_reuses_the_kernel_layer(cluster, lk, proj, "layers-ns")
    finally:
        cluster.stop()


def test_copy_before_the_slow_step_busts_its_cache(tmp_path):
    """The cache keys are real: with the round-4 order (COPY . . first) the kernel-build RUN gets
    a new key on every edit."""
    from devspace_amd.localkube.dockerd import ImageStore, build_image

    store = ImageStore(str(tmp_path / "store"))
    ctx = tmp_path / "ctx"
    (ctx / "devspace_amd").mkdir(parents=True)
    (ctx / "devspace_amd" / "runner.py").write_text("x = 1\n")
    (ctx / "train.py").write_text("v = 1\n")
    (ctx / "Dockerfile").write_text("FROM scratch\nWORKDIR /app\nCOPY . .\nRUN make kernels\nCMD [\"python\"]\n")

    def run_key():
        build_image(store, str(ctx), "Dockerfile", "img:t", log=lambda _: None)
        hist = store.resolve("img:t")["config"]["History"]
        return next(h for h in hist if h["created_by"].startswith("RUN"))

    a = run_key()
    b = run_key()
    assert a["key"] == b["key"] and b["cached"]  # nothing changed: cached
    (ctx / "train.py").write_text("v = 2\n")
    c = run_key()
    assert c["key"] != a["key"] and not c["cached"]
    os.utime(ctx / "train.py", (1, 1))  # an mtime alone is not a change
    d = run_key()
    assert d["key"] == c["key"] and d["cached"]
