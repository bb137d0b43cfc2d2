"""Every record DESIGN.md and profiles/INDEX.md cite is tracked under
profiles/ ("track every trace DESIGN cites"), and every
recipe the runner documents exists."""
import glob
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def expand(cite):
    m = re.search(r"\{([^}]*)\}", cite)
    if not m:
        return [cite]
    out = []
    for alt in m.group(1).split(","):
        out += expand(cite[:m.start()] + alt + cite[m.end():])
    return out


def missing_cites(path, pattern, prefix):
    with open(os.path.join(ROOT, path)) as f:
        text = f.read()
    missing = []
    for cite in sorted(set(re.findall(pattern, text))):
        for c in expand(cite.rstrip(".,)")):
            p = os.path.join(ROOT, prefix, c)
            if not (glob.glob(p) if "*" in p else os.path.exists(p)):
                missing.append(c)
    return missing


def test_design_cites_exist():
    assert missing_cites("DESIGN.md", r"(profiles/[A-Za-z0-9_./{},*\-]+)", "") == []


def test_profiles_index_cites_exist():
    pat = r"`((?:r\d+[a-z0-9_]*/|round6/|pmc_r\w+/)[A-Za-z0-9_./{},*\-]+)`"
    assert missing_cites(os.path.join("profiles", "INDEX.md"), pat, "profiles") == []


def test_gpu_recipes_document_their_recipes():
    path = os.path.join(ROOT, "tools", "gpu_recipes.sh")
    subprocess.check_call(["bash", "-n", path])
    with open(path) as f:
        text = f.read()
    documented = set(re.findall(r"^#   (\w+)\s{2,}", text, re.M))
    implemented = set(re.findall(r"^    (\w+)\)", text, re.M))
    assert documented and documented == implemented, (documented ^ implemented)
