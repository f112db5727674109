"""The native YAML reader against PyYAML (YAML 1.1, like the go-yaml v2 the reference parses
configs and charts with) on mutated copies of the repository's own YAML files: whatever both
accept must read the same, and documents PyYAML accepts must not be rejected (a config the
reference loads must load here). Differences in YAML-1.1-only scalars (`on`/`yes` booleans,
sexagesimal numbers) are normalised away: the rebuild reads YAML 1.2 scalars."""

import glob
import os
import random
import re

import pytest
import yaml

from conftest import ROOT

_native = pytest.importorskip("devspace_amd._native")

YAML11_ONLY = re.compile(r"(?m)(^|[\s:\[{,-])(on|off|yes|no|y|n|On|Off|Yes|No|ON|OFF|YES|NO|Y|N)(\s*:|\s*$|\s*[,\]}])")


def _seeds():
    out = []
    for p in sorted(glob.glob(os.path.join(ROOT, "examples", "**", "*.yaml"), recursive=True)) + sorted(
            glob.glob(os.path.join(ROOT, "tests", "fixtures", "**", "*.yaml"), recursive=True)):
        if os.sep + "templates" + os.sep in p:
            continue
        text = open(p).read()
        try:
            list(yaml.safe_load_all(text))
        except yaml.YAMLError:
            continue
        out.append(text)
    return out


def _norm(v):
    if isinstance(v, dict):
        return {str(k): _norm(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_norm(x) for x in v]
    if isinstance(v, bool) or v is None:
        return v
    if isinstance(v, (int, float)):
        return float(v)
    return v


def test_native_yaml_agrees_with_pyyaml_on_mutations():
    seeds = _seeds()
    assert len(seeds) > 10
    rng = random.Random(20261017)
    alphabet = " \n:-[]{},#'\"ab01."
    agree = 0
    for _ in range(3000):
        s = list(rng.choice(seeds))
        for _ in range(rng.randint(1, 3)):
            i = rng.randrange(len(s))
            op = rng.randint(0, 2)
            if op == 0:
                s[i] = rng.choice(alphabet)
            elif op == 1:
                del s[i:i + rng.randint(1, 6)]
            else:
                s[i:i] = [rng.choice(alphabet) for _ in range(rng.randint(1, 3))]
        text = "".join(s)
        if YAML11_ONLY.search(text):
            continue
        try:
            py = [d for d in yaml.safe_load_all(text) if d is not None]
        except yaml.YAMLError:
            continue
        try:
            ours = [d for d in _native.yaml_parse_all(text) if d is not None]
        except Exception as e:  # noqa: BLE001
            # go-yaml v2 (what the reference parses with) is stricter than PyYAML in two shapes:
            # duplicate mapping keys, and a multi-line plain scalar folded back under a
            # shallower key; tolerated only there
            if "already defined" in str(e) or "indentation" in str(e):
                continue
            raise AssertionError(f"rejected a document PyYAML accepts ({e}):\n{text[:800]}")
        assert [_norm(d) for d in ours] == [_norm(d) for d in py], text[:800]
        agree += 1
    assert agree > 1000


def test_strings_pyyaml_writes_read_back_exactly():
    """What the tests and tools write with yaml.safe_dump and `devspace` then reads: long strings
    with newlines, quotes and runs of spaces come out as double-quoted scalars folded over several
    lines with escaped line breaks (`\\` at the end, `\\ ` for a leading space). An entrypoint
    override carrying a Python program used to gain a space at every fold (an IndentationError in
    the pod)."""
    rng = random.Random(7)
    pieces = ["import os", "\n", "    ", "  ", " ", "x = 1", '"q"', "'s'", "\\", "\t", "#", ": ", "- ", "é", "long" * 7]
    for _ in range(300):
        s = "".join(rng.choice(pieces) for _ in range(rng.randint(1, 60)))
        doc = yaml.safe_dump({"cmd": ["python3", "-c", s], "s": s}, width=rng.choice([40, 80, 120]))
        assert _native.yaml_parse(doc) == {"cmd": ["python3", "-c", s], "s": s}, doc
