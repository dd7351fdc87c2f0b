"""The workshop site (reference Hugo site: config.toml + content/ + layouts/ + static/, SURVEY.md
C01-C04) builds with tools/build_docs.py: every page renders, links resolve, diagrams exist."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_docs_site_builds(tmp_path):
    import build_docs
    out = str(tmp_path / "site")
    pages = build_docs.render(out)
    srcs = {p["rel"] for p in pages}
    assert "_index.md" in srcs and "2_distributed_training/why_how_distributed.md" in srcs
    for name in ("index.html", "404.html", "style.css", "1_setup/index.html", "Appendix/index.html",
                 "2_distributed_training/why_how_distributed.html"):
        assert os.path.isfile(os.path.join(out, name)), name
    for name in ("scale_up_out", "data_parallel", "ps_vs_ring", "xgmi_mesh", "local_flow"):
        svg = open(os.path.join(out, "images", name + ".svg")).read()
        assert svg.startswith("<svg") and svg.rstrip().endswith("</svg>")
    broken = []
    for p in pages:
        page = os.path.join(out, p["out"])
        text = open(page, encoding="utf-8").read()
        assert "{{" not in text, f"unfilled placeholder in {p['out']}"
        assert "<nav" in text or "<ul>" in text
        for url in re.findall(r'(?:href|src)="([^"#]+)', text):
            if re.match(r"^[a-z]+:", url):
                continue
            assert not url.startswith("/"), f"absolute link {url} in {p['out']}"
            target = os.path.normpath(os.path.join(os.path.dirname(page), url))
            if os.path.isdir(target):
                target = os.path.join(target, "index.html")
            if not os.path.exists(target):
                broken.append((p["out"], url))
    # links into the repository tree (e.g. ../../tools/x.py) are allowed to leave the site; only
    # site-internal .html / images / css links must resolve
    broken = [b for b in broken if b[1].endswith((".html", ".svg", ".css"))]
    assert not broken, broken
    concepts = open(os.path.join(out, "2_distributed_training", "why_how_distributed.html")).read()
    assert 'src="../images/xgmi_mesh.svg"' in concepts
    appendix = open(os.path.join(out, "Appendix", "index.html")).read()
    assert 'class="run-local"' in appendix and "build_docs.py" in appendix


def test_docs_notice_shortcode():
    """the learn theme's notice admonitions (reference content uses tip / info / warning)"""
    import build_docs
    from markdown_it import MarkdownIt
    md = MarkdownIt("commonmark", {"html": True})
    out = build_docs._shortcodes("a\n\n{{% notice warning %}}\nNeeds **8** GPUs.\n{{% /notice %}}\n\n"
                                 "{{% notice bogus %}}x{{% /notice %}}", md)
    assert '<div class="notice notice-warning"><p class="notice-title">Warning</p><p>Needs <strong>8</strong>' in out
    assert 'notice notice-note' in out and "{{%" not in out
