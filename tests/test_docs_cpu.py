"""Every measurement the docs cite exists: the `profiles/...` records and the
`tools/...` scripts named in DESIGN.md, README.md, INTEGRATION.md and
tools/README.md (a record split over a line break is matched by its prefix;
`{a,b}` alternatives and `*` globs are expanded)."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ("DESIGN.md", "README.md", "INTEGRATION.md", "tools/README.md")


def _refs(kind):
    out = []
    for doc in DOCS:
        text = open(os.path.join(ROOT, doc)).read()
        for m in re.finditer(kind + r"/([A-Za-z0-9_.*{},\-]+)", text):
            ref = m.group(1).rstrip(".,;:)")
            if not ref:
                continue
            alts = [ref]
            mm = re.match(r"(.*)\{([^}]*)\}(.*)", ref)
            if mm:
                alts = [mm.group(1) + a + mm.group(3) for a in mm.group(2).split(",")]
            out += [(doc, a) for a in alts if "{" not in a]
    return out


def test_cited_profiles_exist():
    missing = [(d, p) for d, p in _refs("profiles")
               if not glob.glob(os.path.join(ROOT, "profiles", p)) and not glob.glob(os.path.join(ROOT, "profiles",
                                                                                                   p + "*"))]
    assert not missing, missing


def test_cited_tools_exist():
    missing = [(d, p) for d, p in _refs("tools")
               if p.endswith((".py", ".sh")) and not glob.glob(os.path.join(ROOT, "tools", p))]
    assert not missing, missing


def test_cited_tests_exist():
    """test functions the docs name (a prefix may stand for a parametrised family)"""
    names = set()
    for f in glob.glob(os.path.join(ROOT, "tests", "*.py")):
        names.update(re.findall(r"^def (test_\w+)", open(f).read(), re.M))
    missing = []
    for doc in DOCS:
        for n in re.findall(r"`(test_\w+)", open(os.path.join(ROOT, doc)).read()):
            if not any(x.startswith(n) for x in names):
                missing.append((doc, n))
    assert not missing, missing
