"""The ctypes mirrors of include/hairpt.h's structs (mitsuba_amd/native.py) have the C
layout: every field at the offset the C compiler gives it, and the same struct size.
A field added to the header but not to the mirror (or in another order) would make
hpt_get_stats / hpt_get_scene_info write past or across the Python structure."""
import ctypes as C
import os
import re
import subprocess

import pytest

from mitsuba_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIRRORS = [("hpt_scene_info", native.SceneInfo), ("hpt_film_params", native.FilmParams),
           ("hpt_render_params", native.RenderParams), ("hpt_stats", native.Stats)]


def _c_layout(tmp_path):
    lines = ["#include <stddef.h>", "#include <stdio.h>", '#include "hairpt.h"', "int main(void) {"]
    for cname, py in MIRRORS:
        lines.append('    printf("%s sizeof %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in py._fields_:
            lines.append('    printf("%s %s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines += ["    return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    out = {}
    for line in subprocess.check_output([str(exe)], text=True).splitlines():
        s, f, v = line.split()
        out[(s, f)] = int(v)
    return out


def test_ctypes_mirrors_match_header(tmp_path):
    c = _c_layout(tmp_path)
    for cname, py in MIRRORS:
        assert C.sizeof(py) == c[(cname, "sizeof")], cname
        for f, _ in py._fields_:
            assert getattr(py, f).offset == c[(cname, f)], (cname, f)


@pytest.mark.parametrize("cname,py", MIRRORS)
def test_every_header_field_is_mirrored(cname, py):
    """Names too: the header's field list (between the typedef and its closing name)
    equals the mirror's."""
    text = open(os.path.join(ROOT, "include", "hairpt.h")).read()
    body = text[text.index("typedef struct %s {" % cname):text.index("} %s;" % cname)]
    names = []
    for stmt in re.sub(r"/\*.*?\*/", "", body, flags=re.S).split(";")[:-1]:
        stmt = stmt.split("{", 1)[-1].strip()
        if not stmt:
            continue
        decl = stmt.split(None, 1)[1] if stmt.split()[0] not in ("unsigned", "const") else stmt.split(None, 2)[2]
        names += [re.sub(r"\[.*\]", "", n).strip().lstrip("*") for n in decl.split(",")]
    assert names == [f for f, _ in py._fields_], cname
