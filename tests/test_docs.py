"""User documentation (docs/): the generated reference pages match the built tool, and every
relative link resolves (reference: docs/pages/** of the original)."""
import glob
import os
import re
import subprocess
import sys

from conftest import ROOT

DOCS = os.path.join(ROOT, "docs")


def test_reference_pages_are_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "gen_docs.py"), "--check"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout


def test_links_resolve_and_every_page_is_indexed():
    pages = sorted(glob.glob(os.path.join(DOCS, "**", "*.md"), recursive=True))
    assert len(pages) >= 10
    for page in pages:
        text = open(page).read()
        for target in re.findall(r"\]\(([^)#\s]+)(?:#[^)]*)?\)", text):
            if re.match(r"[a-z]+://", target):
                continue
            path = os.path.normpath(os.path.join(os.path.dirname(page), target))
            assert os.path.exists(path), f"{os.path.relpath(page, ROOT)}: broken link {target}"
    index = open(os.path.join(DOCS, "README.md")).read()
    for page in pages:
        rel = os.path.relpath(page, DOCS)
        if rel != "README.md":
            assert f"]({rel})" in index, f"docs/README.md does not link {rel}"


def test_every_cli_command_is_in_the_reference():
    text = open(os.path.join(DOCS, "reference", "cli.md")).read()
    for cmd in ("init", "deploy", "dev", "enter", "logs", "analyze", "purge", "reset", "install", "upgrade", "login",
                "add sync", "add package", "create space", "list configs", "remove space", "status sync",
                "update config", "use context"):
        assert f"## `devspace {cmd}`" in text, cmd


def test_every_script_is_a_documented_tool():
    """scripts/ holds only maintained tools: each one has a row in scripts/README.md."""
    readme = open(os.path.join(ROOT, "scripts", "README.md")).read()
    for p in sorted(glob.glob(os.path.join(ROOT, "scripts", "*.py")) + glob.glob(os.path.join(ROOT, "scripts", "*.sh"))):
        assert f"`{os.path.basename(p)}`" in readme, os.path.basename(p)


def test_gpu_tier_passes_only_flags_its_scripts_accept():
    """A GPU-tier step whose flags the script no longer knows fails only on the GPU box: every
    `--flag` passed to bench.py or a scripts/*.py in scripts/gpu_tier.sh is one the script parses."""
    tier = open(os.path.join(ROOT, "scripts", "gpu_tier.sh")).read()
    calls = re.findall(r"python3? -?u? ?\"?(?:\$R/)?((?:scripts/)?\w+\.py)\"?((?:[^\n]|\\\n)*)", tier)
    assert any(c[0] == "bench.py" for c in calls)
    for script, args in calls:
        src = open(os.path.join(ROOT, script)).read()
        for flag in re.findall(r"(?<![\w-])(--[a-z][\w-]*)", args):
            assert f'"{flag}"' in src, f"gpu_tier.sh passes {flag} to {script}, which does not define it"
