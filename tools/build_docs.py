#!/usr/bin/env python
"""Static-site builder for the workshop content in docs/ (the reference serves its content with
Hugo and the "learn" theme: config.toml, content/, layouts/, themes/, static/ -- SURVEY.md C01-C04;
Hugo is not available here, so this renders the same kind of site with the Python standard library
plus markdown-it).

    python tools/build_docs.py --out /tmp/site

* ``docs/site.toml``: title, author, menu titles of the sections, concept diagrams;
* ``docs/**/*.md``: pages (optional ``---`` front matter with ``title`` / ``weight``); a section is a
  numbered directory with an ``_index.md``;
* ``docs/layouts/{page,404}.html``: the page shell ({{menu}}, {{content}}, ... placeholders);
* ``docs/static/``: copied as-is;
* concept slides (reference ``static/images/training/training21-24.png``) are drawn as SVG from
  code, written to ``<out>/images/``, and referenced from pages as ``/images/<name>.svg``;
* ``docs/layouts/partials/*.html``: header / menu / toc / footer pieces, included by
  ``{{partial "name"}}`` (the reference's ``layouts/partials``);
* shortcodes (the reference's ``layouts/shortcodes``): ``{{< run-local cmd="..." >}}`` renders a
  "run it locally" box, and so do ``cf-launch`` / ``cf-download`` (the reference's CloudFormation
  buttons: there is no AWS account to launch into -- the box names the local command instead);
  ``{{< tabs >}}{{< tab name="..." >}}...{{< /tab >}}{{< /tabs >}}`` renders a tab set (CSS radio
  tabs, no JavaScript); ``{{< mermaid >}}...{{< /mermaid >}}`` keeps the diagram source in a
  ``<pre class="mermaid">`` block (rendered by mermaid.js where a page loads it, readable as text
  otherwise); ``{{< year >}}`` and ``{{< github repo="..." >}}``; ``{{% notice tip|info|note|warning %}}
  ...{{% /notice %}}`` renders a coloured admonition with a markdown body;
* a table of contents per page from its ``##`` / ``###`` headings (the reference's ``toc`` partial);
* links: ``x.md`` -> ``x.html`` and root-relative ``/...`` made page-relative (``relative_urls``).
"""
from __future__ import annotations

import argparse
import html
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = os.path.join(ROOT, "docs")


# ----------------------------------------------------------------------------- diagrams
def _svg(w, h, body, title):
    return (f'<svg xmlns="http://www.w3.org/2000/svg" width="{w}" height="{h}" viewBox="0 0 {w} {h}" '
            f'font-family="Helvetica, Arial, sans-serif" font-size="13">\n<title>{html.escape(title)}</title>\n'
            '<defs><marker id="a" markerWidth="8" markerHeight="8" refX="7" refY="4" orient="auto">'
            '<path d="M0,0 L8,4 L0,8 z" fill="#333"/></marker></defs>\n' + body + "\n</svg>\n")


def _box(x, y, w, h, label, fill="#dbe9ff"):
    lines = label.split("\n")
    t = "".join(f'<tspan x="{x + w / 2}" dy="{0 if i == 0 else 15}">{html.escape(s)}</tspan>'
                for i, s in enumerate(lines))
    ty = y + h / 2 - 7 * (len(lines) - 1) + 4
    return (f'<rect x="{x}" y="{y}" width="{w}" height="{h}" rx="6" fill="{fill}" stroke="#335"/>'
            f'<text x="{x + w / 2}" y="{ty}" text-anchor="middle">{t}</text>')


def _arrow(x1, y1, x2, y2, label=""):
    s = f'<line x1="{x1}" y1="{y1}" x2="{x2}" y2="{y2}" stroke="#333" marker-end="url(#a)"/>'
    if label:
        s += f'<text x="{(x1 + x2) / 2 + 4}" y="{(y1 + y2) / 2 - 4}" font-size="11">{html.escape(label)}</text>'
    return s


def _text(x, y, s, size=13, anchor="start"):
    return f'<text x="{x}" y="{y}" font-size="{size}" text-anchor="{anchor}">{html.escape(s)}</text>'


def diagram_scale_up_out(title):
    b = [_text(20, 24, "Scale up: one bigger device", 14), _box(40, 40, 220, 90, "1 x MI355X\n288 GB HBM3E\n~2.5 PFLOP/s bf16")]
    b.append(_text(330, 24, "Scale out: more devices on one job", 14))
    for i in range(8):
        b.append(_box(330 + (i % 4) * 80, 40 + (i // 4) * 50, 70, 40, f"GPU {i}", "#e4f5e1"))
    b.append(_text(330, 160, "8 x MI355X, fully connected by xGMI", 12))
    return _svg(660, 180, "\n".join(b), title)


def diagram_data_parallel(title):
    b = [_box(250, 10, 160, 40, "global batch 256")]
    for i in range(4):
        x = 30 + i * 160
        b += [_arrow(330, 50, x + 60, 90), _box(x, 90, 120, 40, f"rank {i}: 64 images"),
              _arrow(x + 60, 130, x + 60, 160), _box(x, 160, 120, 40, "fwd + bwd\n(model replica)", "#e4f5e1"),
              _arrow(x + 60, 200, x + 60, 230)]
    b.append(_box(30, 230, 600, 36, "all-reduce: average the gradients (every replica gets the same update)", "#ffe9cc"))
    return _svg(660, 280, "\n".join(b), title)


def diagram_ps_vs_ring(title):
    b = [_text(20, 22, "Parameter server: every gradient crosses the server's links", 13),
         _box(120, 35, 120, 36, "server", "#ffe9cc")]
    for i in range(4):
        x = 20 + i * 90
        b += [_box(x, 120, 70, 34, f"worker {i}"), _arrow(x + 35, 120, 180, 71)]
    b.append(_text(420, 22, "Ring all-reduce: 2(N-1)/N of the data per link", 13))
    import math
    cx, cy, r = 560, 100, 60
    for i in range(4):
        a = 2 * math.pi * i / 4 - math.pi / 2
        x, y = cx + r * math.cos(a), cy + r * math.sin(a)
        a2 = 2 * math.pi * (i + 1) / 4 - math.pi / 2
        x2, y2 = cx + r * math.cos(a2), cy + r * math.sin(a2)
        b.append(_arrow(x + (x2 - x) * 0.25, y + (y2 - y) * 0.25, x + (x2 - x) * 0.75, y + (y2 - y) * 0.75))
        b.append(_box(x - 30, y - 15, 60, 30, f"GPU {i}", "#e4f5e1"))
    return _svg(700, 180, "\n".join(b), title)


def diagram_xgmi_mesh(title):
    b = [_text(20, 20, "SMDDP: fusion buffer split into N balanced shards", 13)]
    for i in range(8):
        b.append(_box(20 + i * 60, 30, 56, 30, f"shard {i}", "#ffe9cc"))
    b.append(_text(20, 90, "MI355X: every GPU reduces ITS shard from all 7 peers over 7 xGMI links at once", 13))
    b.append(_text(20, 106, "(reduce-scatter), then all-gathers the reduced shards -- csrc/kernels/ipc_allreduce.hip", 12))
    import math
    cx, cy, r = 250, 230, 95
    pts = []
    for i in range(8):
        a = 2 * math.pi * i / 8
        pts.append((cx + r * math.cos(a), cy + r * math.sin(a)))
    for i in range(8):
        for j in range(i + 1, 8):
            b.append(f'<line x1="{pts[i][0]:.1f}" y1="{pts[i][1]:.1f}" x2="{pts[j][0]:.1f}" y2="{pts[j][1]:.1f}" '
                     'stroke="#9ab" stroke-width="1"/>')
    for i, (x, y) in enumerate(pts):
        b.append(_box(x - 26, y - 14, 52, 28, f"GPU {i}", "#e4f5e1"))
    b.append(_text(390, 200, "7 links x ~153 GB/s per GPU", 12))
    b.append(_text(390, 220, "ring: one link per direction", 12))
    b.append(_text(390, 240, "mesh RS/AG: all 7 links", 12))
    return _svg(620, 350, "\n".join(b), title)


def diagram_local_flow(title):
    steps = ["notebook\nPyTorch(...).fit()", "local job runner\nSM_* env, model.tar.gz", "mi355x_launch\n1 rank / GPU",
             "user script\nDDP over smddp", "deploy / predict\nmodel_fn"]
    b = []
    for i, s in enumerate(steps):
        x = 10 + i * 140
        b.append(_box(x, 30, 125, 50, s, "#dbe9ff" if i % 2 == 0 else "#e4f5e1"))
        if i:
            b.append(_arrow(x - 15, 55, x, 55))
    return _svg(720, 100, "\n".join(b), title)


DIAGRAMS = {"scale_up_out": diagram_scale_up_out, "data_parallel": diagram_data_parallel,
            "ps_vs_ring": diagram_ps_vs_ring, "xgmi_mesh": diagram_xgmi_mesh, "local_flow": diagram_local_flow}


# ------------------------------------------------------------------------------- pages
def _front_matter(text):
    meta = {}
    if text.startswith("---\n"):
        end = text.find("\n---", 4)
        if end > 0:
            for line in text[4:end].splitlines():
                if ":" in line:
                    k, v = line.split(":", 1)
                    meta[k.strip()] = v.strip().strip('"').strip()
            text = text[end + 4:].lstrip("\n")
    return meta, text


def _title(meta, text, fallback):
    if meta.get("title"):
        return meta["title"]
    m = re.search(r"^#\s+(.+)$", text, re.M)
    return m.group(1).strip() if m else fallback


def _rel(from_page, target):
    """page-relative link from the output file ``from_page`` (posix, relative to the site root)"""
    depth = from_page.count("/")
    return "../" * depth + target.lstrip("/")


def _run_local_box(cmd):
    return f'<div class="run-local"><strong>Run locally</strong><pre><code>{html.escape(cmd)}</code></pre></div>'


_TABSET = [0]
# the learn theme's ``{{% notice <kind> %}}...{{% /notice %}}`` admonitions (reference content uses
# tip / info / warning, e.g. content/2_distributed_training/pytorch_smddp_dist_training.md:6-20)
_NOTICE_KINDS = {"note": "Note", "info": "Info", "tip": "Tip", "warning": "Warning"}


def _shortcodes(text, md=None):
    """Expand the shortcodes (module docstring) before markdown rendering; tab bodies are rendered
    as markdown themselves (``md``)."""
    text = re.sub(r'\{\{<\s*run-local\s+cmd="([^"]*)"\s*>\}\}', lambda m: _run_local_box(m.group(1)), text)
    # CloudFormation buttons of the reference -> the local command of the same step
    text = re.sub(r'\{\{<\s*cf-(?:launch|download)\s+([^>]*)>\}\}',
                  lambda m: _run_local_box(re.search(r'cmd="([^"]*)"', m.group(1)).group(1)
                                           if 'cmd="' in m.group(1) else "python -m mi355x_dp.launch --help"), text)
    text = re.sub(r'\{\{<\s*year\s*>\}\}', lambda m: str(__import__("datetime").date.today().year), text)
    text = re.sub(r'\{\{<\s*github\s+repo="([^"]*)"\s*>\}\}',
                  lambda m: f'<a class="github" href="https://github.com/{html.escape(m.group(1))}">'
                            f'{html.escape(m.group(1))}</a>', text)

    def notice(m):
        kind = m.group(1) if m.group(1) in _NOTICE_KINDS else "note"
        inner = md.render(m.group(2).strip()) if md is not None else html.escape(m.group(2).strip())
        return f'<div class="notice notice-{kind}"><p class="notice-title">{_NOTICE_KINDS[kind]}</p>{inner}</div>'
    text = re.sub(r'\{\{%\s*notice\s+(\w+)\s*%\}\}(.*?)\{\{%\s*/notice\s*%\}\}', notice, text, flags=re.S)

    def mermaid(m):
        return f'<pre class="mermaid">{html.escape(m.group(1).strip())}</pre>'
    text = re.sub(r'\{\{<\s*mermaid\s*>\}\}(.*?)\{\{<\s*/mermaid\s*>\}\}', mermaid, text, flags=re.S)

    def tabs(m):
        _TABSET[0] += 1
        sid = f"tabset-{_TABSET[0]}"
        items = re.findall(r'\{\{<\s*tab\s+name="([^"]*)"\s*>\}\}(.*?)\{\{<\s*/tab\s*>\}\}', m.group(1), flags=re.S)
        out = [f'<div class="tabs" id="{sid}">']
        for i, (name, body) in enumerate(items):
            tid = f"{sid}-{i}"
            inner = md.render(body.strip()) if md is not None else html.escape(body.strip())
            out.append(f'<input type="radio" name="{sid}" id="{tid}"{" checked" if i == 0 else ""}>'
                       f'<label for="{tid}">{html.escape(name.strip())}</label>'
                       f'<div class="tab-body">{inner}</div>')
        out.append("</div>")
        return "".join(out)
    return re.sub(r'\{\{<\s*tabs[^>]*>\}\}(.*?)\{\{<\s*/tabs\s*>\}\}', tabs, text, flags=re.S)


def _toc(body_html):
    """table of contents from the rendered page's h2 / h3 headings (ids added in place)"""
    heads = []

    def anchor(m):
        level, inner = m.group(1), m.group(2)
        text = re.sub(r"<[^>]+>", "", inner)
        slug = re.sub(r"[^a-z0-9]+", "-", text.lower()).strip("-") or f"h{len(heads)}"
        heads.append((int(level), slug, text))
        return f'<h{level} id="{slug}">{inner}</h{level}>'
    body_html = re.sub(r"<h([23])>(.*?)</h\1>", anchor, body_html)
    if not heads:
        return body_html, ""
    items = "".join(f'<li class="toc-h{lv}"><a href="#{slug}">{t}</a></li>' for lv, slug, t in heads)
    return body_html, f"<ul>{items}</ul>"


def collect(docs=DOCS):
    pages = []
    for dirpath, dirnames, filenames in os.walk(docs):
        rel_dir = os.path.relpath(dirpath, docs)
        if rel_dir.split(os.sep)[0] in ("layouts", "static"):
            continue
        dirnames.sort()
        for f in sorted(filenames):
            if not f.endswith(".md"):
                continue
            src = os.path.join(dirpath, f)
            meta, text = _front_matter(open(src, encoding="utf-8").read())
            rel = os.path.relpath(src, docs).replace(os.sep, "/")
            out = "index.html" if rel == "_index.md" else re.sub(r"_index\.md$", "index.html", rel)
            out = re.sub(r"\.md$", ".html", out)
            section = rel.split("/")[0] if "/" in rel else ""
            pages.append({"src": src, "rel": rel, "out": out, "section": section, "meta": meta, "text": text,
                          "title": _title(meta, text, f), "weight": float(meta.get("weight", 0 if f == "_index.md" else 50))})
    return pages


def _menu(pages, cfg, current):
    order = lambda s: (int(m.group(1)) if (m := re.match(r"(\d+)", s)) else 99, s)  # noqa: E731
    sections = sorted({p["section"] for p in pages if p["section"]}, key=order)
    items = [f'<li class="{"active" if current == "index.html" else ""}"><a href="{_rel(current, "index.html")}">Home</a></li>']
    for sec in sections:
        sp = sorted([p for p in pages if p["section"] == sec], key=lambda p: (p["weight"], p["rel"]))
        head = next((p for p in sp if p["rel"].endswith("_index.md")), sp[0])
        title = cfg.get("menu", {}).get(sec, head["title"])
        sub = "".join(f'<li class="{"active" if p["out"] == current else ""}"><a href="{_rel(current, p["out"])}">'
                      f'{html.escape(p["title"])}</a></li>' for p in sp if p is not head)
        items.append(f'<li class="{"active" if head["out"] == current else ""}"><a href="{_rel(current, head["out"])}">'
                     f'{html.escape(title)}</a>{f"<ul>{sub}</ul>" if sub else ""}</li>')
    return "<ul>" + "".join(items) + "</ul>"


def render(out_dir, docs=DOCS):
    import tomli
    from markdown_it import MarkdownIt
    cfg = tomli.load(open(os.path.join(docs, "site.toml"), "rb"))
    md = MarkdownIt("commonmark", {"html": True}).enable("table")
    layout = open(os.path.join(docs, "layouts", "page.html"), encoding="utf-8").read()
    pdir = os.path.join(docs, "layouts", "partials")
    for name in sorted(os.listdir(pdir)) if os.path.isdir(pdir) else []:
        if name.endswith(".html"):
            part = open(os.path.join(pdir, name), encoding="utf-8").read().strip()
            layout = layout.replace('{{partial "' + name[:-5] + '"}}', part)
    if os.path.exists(out_dir):
        shutil.rmtree(out_dir)
    shutil.copytree(os.path.join(docs, "static"), out_dir)
    os.makedirs(os.path.join(out_dir, "images"), exist_ok=True)
    for name, title in cfg.get("diagrams", {}).items():
        with open(os.path.join(out_dir, "images", f"{name}.svg"), "w", encoding="utf-8") as f:
            f.write(DIAGRAMS[name](title))
    pages = collect(docs)
    for p in pages:
        body, toc = _toc(md.render(_shortcodes(p["text"], md)))
        cur = p["out"]

        def fix(m, cur=cur):
            attr, url = m.group(1), m.group(2)
            if re.match(r"^[a-z]+:", url) or url.startswith("#"):
                return m.group(0)
            url = re.sub(r"_index\.md(#|$)", r"index.html\1", url)
            url = re.sub(r"\.md(#|$)", r".html\1", url)
            if url.startswith("/"):
                url = _rel(cur, url)
            return f'{attr}="{url}"'

        body = re.sub(r'(href|src)="([^"]*)"', fix, body)
        page = layout
        for k, v in (("language", cfg.get("language", "en")), ("description", cfg.get("description", "")),
                     ("author", cfg.get("author", "")), ("site_title", cfg["title"]), ("title", p["title"]),
                     ("root", _rel(cur, "")), ("menu", _menu(pages, cfg, cur)), ("toc", toc),
                     ("year", str(__import__("datetime").date.today().year)), ("content", body)):
            page = page.replace("{{" + k + "}}", html.escape(v) if k in ("title", "site_title", "description", "author") else v)
        dst = os.path.join(out_dir, cur)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        with open(dst, "w", encoding="utf-8") as f:
            f.write(page)
    nf = open(os.path.join(docs, "layouts", "404.html"), encoding="utf-8").read()
    for k, v in (("language", cfg.get("language", "en")), ("site_title", html.escape(cfg["title"])), ("root", "")):
        nf = nf.replace("{{" + k + "}}", v)
    with open(os.path.join(out_dir, "404.html"), "w", encoding="utf-8") as f:
        f.write(nf)
    return pages


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "build", "site"))
    a = ap.parse_args(argv)
    pages = render(a.out)
    print(f"[docs] {len(pages)} pages -> {a.out}/index.html")
    return 0


if __name__ == "__main__":
    sys.exit(main())
