"""What travels to the GPU box and what the product may touch (CPU).

oracle/_ref/ (the reference's own objects built from /root/reference:
nsref, libnsdrefip.so) is git-ignored but NOT gpurun-ignored: it travels
with the tree so that bench.py's cpu_baseline can time the reference harness
on the GPU box's host cores (`reference_harness_1thread` /
`reference_harness_all_cores`).  Nothing else there may use it:

* no product file under netsniff-ng_amd/ names the oracle or the reference
  build in code (comments citing the oracle as a model are allowed), and the
  product library neither links nor names either;
* no `-m gpu` test reaches oracle/_ref, directly or through a helper of its
  own module or of nsd_testlib (the GPU tests check against the oracle
  restatement and the committed goldens, which the reference build made
  here).
"""
import ast
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "netsniff-ng_amd")
FORBIDDEN = re.compile(r"oracle/_ref|_ref/|\bnsref\b|nsref_|REF_BIN|REF_IP_SO|HAVE_REF|run_ref|libnsdrefip|"
                       r"libnsdoracle|\bnsor_")
# the GPU tests may use the oracle restatement (nsor_*), never the reference build
REF_BUILD = re.compile(r"oracle/_ref|_ref/|\bnsref\b|nsref_|REF_BIN|REF_IP_SO|HAVE_REF|run_ref|libnsdrefip")
# nsd_testlib helpers that run or load oracle/_ref
TESTLIB_REF = {"run_ref", "REF_BIN"}


def _strip_comments(path, text):
    if path.endswith(".py"):
        out = []
        for line in text.splitlines():
            s = line.split("#", 1)[0]
            out.append(s)
        text = "\n".join(out)
        return re.sub(r'"""(.*?)"""', "", text, flags=re.S)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    return re.sub(r"(?m)^\s*#\s*(?!include|define|if|ifdef|ifndef|else|endif|pragma|undef).*$", "", text)


def test_product_sources_never_name_the_oracle_or_reference_build():
    bad = []
    for d, _, files in os.walk(PKG):
        if "__pycache__" in d or os.sep + "build" in d:
            continue
        for fn in files:
            if not fn.endswith((".py", ".hip", ".cpp", ".h", ".c")) and fn != "Makefile":
                continue
            p = os.path.join(d, fn)
            with open(p, errors="replace") as f:
                code = _strip_comments(p, f.read())
            for m in FORBIDDEN.finditer(code):
                bad.append(f"{os.path.relpath(p, ROOT)}: {m.group(0)}")
            if re.search(r"\boracle\b", code):
                bad.append(f"{os.path.relpath(p, ROOT)}: oracle")
    assert not bad, bad


def test_product_library_links_neither():
    so = os.path.join(PKG, "libnsdissect.so")
    if not os.path.exists(so):
        pytest.skip("product library not built")
    r = subprocess.run(["readelf", "-d", so], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
    needed = re.findall(r"\(NEEDED\)\s+Shared library: \[(.*?)\]", r.stdout)
    assert needed and not [n for n in needed if "oracle" in n or "nsdref" in n or "nsdoracle" in n], needed
    with open(so, "rb") as f:
        blob = f.read()
    for s in (b"libnsdoracle", b"libnsdrefip", b"oracle/_ref", b"nsor_dissect"):
        assert s not in blob, s


def _is_gpu_mark(node):
    return isinstance(node, ast.Attribute) and node.attr == "gpu" or \
        isinstance(node, ast.Call) and _is_gpu_mark(node.func)


def _module_gpu(tree):
    for st in tree.body:
        if isinstance(st, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "pytestmark" for t in st.targets):
            v = st.value
            items = v.elts if isinstance(v, (ast.List, ast.Tuple)) else [v]
            if any(_is_gpu_mark(x) for x in items):
                return True
    return False


def _names_used(fn):
    out = set()
    for n in ast.walk(fn):
        if isinstance(n, ast.Name):
            out.add(n.id)
        elif isinstance(n, ast.Attribute):
            out.add(n.attr)
    return out


def test_gpu_tests_never_reach_the_reference_build():
    tests = os.path.join(ROOT, "tests")
    checked, bad = 0, []
    for fn in sorted(os.listdir(tests)):
        if not (fn.startswith("test_") and fn.endswith(".py")):
            continue
        path = os.path.join(tests, fn)
        with open(path) as f:
            src = f.read()
        tree = ast.parse(src)
        funcs = {st.name: st for st in tree.body if isinstance(st, ast.FunctionDef)}
        mod_gpu = _module_gpu(tree)
        for name, node in funcs.items():
            if not name.startswith("test_"):
                continue
            if not (mod_gpu or any(_is_gpu_mark(dec) for dec in node.decorator_list)):
                continue
            checked += 1
            # the test body and every module function it reaches (decorators
            # excluded: a skipif on the reference build is not a use of it)
            seen, todo = set(), [name]
            while todo:
                f = todo.pop()
                if f in seen:
                    continue
                seen.add(f)
                fnode = funcs[f]
                stmts = [st for st in fnode.body   # (docstrings may cite the goldens' origin)
                         if not (isinstance(st, ast.Expr) and isinstance(st.value, ast.Constant))]
                used = _names_used(ast.Module(body=stmts, type_ignores=[]))
                seg = "\n".join(ast.get_source_segment(src, st) or "" for st in stmts)
                for m in REF_BUILD.finditer(seg):
                    bad.append(f"{fn}::{name} via {f}: {m.group(0)}")
                for u in used & TESTLIB_REF:
                    bad.append(f"{fn}::{name} via {f}: T.{u}")
                todo.extend(u for u in used if u in funcs and u not in seen)
    assert checked >= 40, checked   # 43 GPU test functions (221 cases): the scan must have seen them
    assert not bad, bad
