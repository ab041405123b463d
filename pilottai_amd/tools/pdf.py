"""Dependency-free PDF text extraction (and a tiny writer for tests/examples).

Replaces the `pypdf` dependency of the reference example
(docs/examples/pdf_processing/pdf_extractor.py:1-40), which is not available
here. Supports what ordinary generated PDFs use:

* classic xref tables and PDF 1.5 object streams (/Type /ObjStm),
* /FlateDecode streams (zlib), page-tree traversal in document order,
* simple fonts (1-byte codes, WinAnsi/standard ~ latin-1) and Type0 / Identity-H
  CID fonts (2-byte codes) with /ToUnicode CMaps (bfchar + bfrange),
* text operators Tj, TJ, ', " with Td / TD / Tm / T* positioning: a change of
  baseline starts a new line, a wide horizontal gap inserts a space.

It is not a renderer: no glyph-width metrics, no encryption, no LZW/JBIG2.
"""
from __future__ import annotations

import re
import zlib
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

# --------------------------------------------------------------------------- lexer / parser


@dataclass(frozen=True)
class Ref:
    num: int
    gen: int = 0


class Name(str):
    pass


class Op(bytes):
    """A bare keyword / content-stream operator (strings are plain bytes)."""


_WS = b" \t\r\n\x00\x0c"
_DELIM = b"()<>[]{}/%"


class _Parser:
    def __init__(self, data: bytes, pos: int = 0):
        self.d = data
        self.p = pos

    def skip(self):
        d, n = self.d, len(self.d)
        while self.p < n:
            c = d[self.p]
            if c in _WS:
                self.p += 1
            elif c == 0x25:  # % comment
                while self.p < n and d[self.p] not in b"\r\n":
                    self.p += 1
            else:
                break

    def token(self) -> bytes:
        self.skip()
        d, s = self.d, self.p
        while self.p < len(d) and d[self.p] not in _WS and d[self.p] not in _DELIM:
            self.p += 1
        return d[s:self.p]

    def obj(self) -> Any:
        self.skip()
        d = self.d
        if self.p >= len(d):
            raise EOFError
        c = d[self.p:self.p + 1]
        if c == b"<":
            if d[self.p + 1:self.p + 2] == b"<":
                self.p += 2
                out: Dict[str, Any] = {}
                while True:
                    self.skip()
                    if d[self.p:self.p + 2] == b">>":
                        self.p += 2
                        return out
                    key = self.obj()
                    out[str(key)] = self.obj()
            self.p += 1
            e = d.index(b">", self.p)
            hx = re.sub(rb"\s", b"", d[self.p:e])
            self.p = e + 1
            if len(hx) % 2:
                hx += b"0"
            return bytes.fromhex(hx.decode())
        if c == b"[":
            self.p += 1
            arr = []
            while True:
                self.skip()
                if d[self.p:self.p + 1] == b"]":
                    self.p += 1
                    return arr
                arr.append(self.obj())
        if c == b"(":
            return self._literal()
        if c == b"/":
            self.p += 1
            t = self.token()
            return Name(re.sub(rb"#([0-9a-fA-F]{2})", lambda m: bytes([int(m.group(1), 16)]), t).decode("latin-1"))
        t = self.token()
        if not t:
            self.p += 1
            return None
        if re.fullmatch(rb"[+-]?\d+", t):
            # lookahead for "gen R"
            save = self.p
            t2 = self.token()
            if re.fullmatch(rb"\d+", t2 or b""):
                t3 = self.token()
                if t3 == b"R":
                    return Ref(int(t), int(t2))
            self.p = save
            return int(t)
        if re.fullmatch(rb"[+-]?(\d+\.\d*|\.\d+|\d+)", t):
            return float(t)
        if t == b"true":
            return True
        if t == b"false":
            return False
        if t == b"null":
            return None
        return Op(t)  # operator / keyword

    def _literal(self) -> bytes:
        d = self.d
        self.p += 1
        out = bytearray()
        depth = 1
        esc = {ord("n"): 10, ord("r"): 13, ord("t"): 9, ord("b"): 8, ord("f"): 12}
        while self.p < len(d):
            c = d[self.p]
            self.p += 1
            if c == 0x5C:  # backslash
                n = d[self.p]
                self.p += 1
                if n in esc:
                    out.append(esc[n])
                elif 0x30 <= n <= 0x37:
                    oct_ = bytes([n])
                    while len(oct_) < 3 and 0x30 <= d[self.p] <= 0x37:
                        oct_ += bytes([d[self.p]])
                        self.p += 1
                    out.append(int(oct_, 8) & 0xFF)
                elif n in b"\r\n":
                    if n == 0x0D and d[self.p:self.p + 1] == b"\n":
                        self.p += 1
                else:
                    out.append(n)
            elif c == 0x28:
                depth += 1
                out.append(c)
            elif c == 0x29:
                depth -= 1
                if depth == 0:
                    break
                out.append(c)
            else:
                out.append(c)
        return bytes(out)


# --------------------------------------------------------------------------- document


class PDFDocument:
    def __init__(self, data: bytes):
        if not data.startswith(b"%PDF"):
            raise ValueError("not a PDF file")
        self.data = data
        self.objects: Dict[int, Any] = {}
        self.streams: Dict[int, bytes] = {}
        self._scan()
        self._expand_object_streams()

    # raw object scan (robust to broken xref tables)
    def _scan(self):
        d = self.data
        for m in re.finditer(rb"(\d+)\s+(\d+)\s+obj\b", d):
            num = int(m.group(1))
            p = _Parser(d, m.end())
            try:
                o = p.obj()
            except Exception:  # noqa: BLE001 — skip unparsable objects
                continue
            p.skip()
            if isinstance(o, dict) and d.startswith(b"stream", p.p):
                s = p.p + 6
                if d[s:s + 2] == b"\r\n":
                    s += 2
                elif d[s:s + 1] in (b"\n", b"\r"):
                    s += 1
                ln = o.get("Length")
                e = s + ln if isinstance(ln, int) and d.startswith(b"endstream", self._skipws(s + ln)) \
                    else d.find(b"endstream", s)
                self.streams[num] = d[s:e]
            self.objects[num] = o

    def _skipws(self, i: int) -> int:
        while i < len(self.data) and self.data[i] in _WS:
            i += 1
        return i

    def resolve(self, o: Any) -> Any:
        seen = 0
        while isinstance(o, Ref) and seen < 32:
            o = self.objects.get(o.num)
            seen += 1
        return o

    def stream(self, ref_or_num) -> bytes:
        num = ref_or_num.num if isinstance(ref_or_num, Ref) else int(ref_or_num)
        raw = self.streams.get(num, b"")
        dic = self.objects.get(num) or {}
        filt = self.resolve(dic.get("Filter"))
        filters = filt if isinstance(filt, list) else ([filt] if filt else [])
        for f in filters:
            f = self.resolve(f)
            if f in ("FlateDecode", "Fl"):
                try:
                    raw = zlib.decompress(raw)
                except zlib.error:
                    raw = zlib.decompressobj().decompress(raw)
                parms = self.resolve(dic.get("DecodeParms")) or {}
                if isinstance(parms, dict) and int(parms.get("Predictor", 1) or 1) >= 10:
                    raw = _png_unpredict(raw, int(parms.get("Columns", 1) or 1))
            else:
                raise ValueError(f"unsupported PDF stream filter {f}")
        return raw

    def _expand_object_streams(self):
        for num, o in list(self.objects.items()):
            if not (isinstance(o, dict) and o.get("Type") == "ObjStm"):
                continue
            data = self.stream(num)
            n, first = int(o.get("N", 0)), int(o.get("First", 0))
            hdr = _Parser(data[:first])
            pairs = []
            for _ in range(n):
                pairs.append((int(hdr.obj()), int(hdr.obj())))
            for onum, off in pairs:
                if onum in self.objects:
                    continue
                try:
                    self.objects[onum] = _Parser(data, first + off).obj()
                except Exception:  # noqa: BLE001
                    pass

    def pages(self) -> List[dict]:
        root = None
        for o in self.objects.values():
            if isinstance(o, dict) and o.get("Type") == "Catalog":
                root = o
                break
        out: List[dict] = []

        def walk(node, inherited):
            node = self.resolve(node)
            if not isinstance(node, dict):
                return
            res = node.get("Resources", inherited)
            if node.get("Type") == "Pages" or "Kids" in node:
                for k in self.resolve(node.get("Kids")) or []:
                    walk(k, res)
            else:
                page = dict(node)
                page.setdefault("Resources", res)
                out.append(page)

        if root is not None and root.get("Pages") is not None:
            walk(root["Pages"], None)
        if not out:  # no usable page tree: every /Page in file order
            out = [o for o in self.objects.values() if isinstance(o, dict) and o.get("Type") == "Page"]
        return out


def _png_unpredict(data: bytes, columns: int) -> bytes:
    row = columns + 1
    out = bytearray()
    prev = bytearray(columns)
    for i in range(0, len(data), row):
        ft, line = data[i], bytearray(data[i + 1:i + row])
        for j in range(len(line)):
            a = line[j - 1] if j else 0
            if ft == 2:
                line[j] = (line[j] + prev[j]) & 0xFF
            elif ft == 1:
                line[j] = (line[j] + a) & 0xFF
            elif ft == 3:
                line[j] = (line[j] + ((a + prev[j]) >> 1)) & 0xFF
            elif ft == 4:
                b, c = prev[j], (prev[j - 1] if j else 0)
                pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                line[j] = (line[j] + (a if pa <= pb and pa <= pc else b if pb <= pc else c)) & 0xFF
        out += line
        prev = line
    return bytes(out)


# --------------------------------------------------------------------------- fonts


class _Font:
    def __init__(self, doc: PDFDocument, font: dict):
        self.two_byte = font.get("Subtype") == "Type0"
        self.cmap: Dict[int, str] = {}
        tu = font.get("ToUnicode")
        if isinstance(tu, Ref):
            try:
                self._parse_cmap(doc.stream(tu))
            except Exception:  # noqa: BLE001 — fall back to raw codes
                pass

    def _parse_cmap(self, data: bytes):
        for block in re.findall(rb"beginbfchar(.*?)endbfchar", data, re.S):
            for src, dst in re.findall(rb"<([0-9a-fA-F]+)>\s*<([0-9a-fA-F]*)>", block):
                self.cmap[int(src, 16)] = _utf16(dst)
        for block in re.findall(rb"beginbfrange(.*?)endbfrange", data, re.S):
            for m in re.finditer(rb"<([0-9a-fA-F]+)>\s*<([0-9a-fA-F]+)>\s*(\[[^\]]*\]|<[0-9a-fA-F]*>)", block):
                lo, hi, dst = int(m.group(1), 16), int(m.group(2), 16), m.group(3)
                if dst.startswith(b"["):
                    for i, h in enumerate(re.findall(rb"<([0-9a-fA-F]*)>", dst)):
                        self.cmap[lo + i] = _utf16(h)
                else:
                    base = int(dst[1:-1] or b"0", 16)
                    for i in range(hi - lo + 1):
                        self.cmap[lo + i] = chr(base + i) if base + i < 0x110000 else ""

    def decode(self, s: bytes) -> str:
        if self.two_byte:
            codes = [int.from_bytes(s[i:i + 2], "big") for i in range(0, len(s) - 1, 2)]
        else:
            codes = list(s)
        if self.cmap:
            return "".join(self.cmap.get(c, "") for c in codes)
        return "".join(chr(c) if c < 0x110000 else "" for c in codes)


def _utf16(hexstr: bytes) -> str:
    try:
        return bytes.fromhex(hexstr.decode()).decode("utf-16-be", errors="ignore")
    except ValueError:
        return ""


# --------------------------------------------------------------------------- content streams


def _page_text(doc: PDFDocument, page: dict) -> str:
    res = doc.resolve(page.get("Resources")) or {}
    fonts_d = doc.resolve(res.get("Font")) if isinstance(res, dict) else None
    fonts: Dict[str, _Font] = {}
    if isinstance(fonts_d, dict):
        for name, ref in fonts_d.items():
            f = doc.resolve(ref)
            if isinstance(f, dict):
                fonts[name] = _Font(doc, f)
    contents = page.get("Contents")
    parts = contents if isinstance(contents, list) else [contents]
    data = b"\n".join(doc.stream(p) for p in parts if isinstance(p, Ref))
    ps = _Parser(data)
    ops: List[Any] = []
    out: List[str] = []
    font: Optional[_Font] = None
    size = 12.0
    line_y: Optional[float] = None
    x = y = 0.0           # current text line start (text space, before the CTM)
    last_x_end: Optional[float] = None

    def emit(txt: str, at_x: float, at_y: float):
        nonlocal line_y, last_x_end
        if line_y is not None and abs(at_y - line_y) > 0.5 * max(size, 1.0):
            out.append("\n")
            last_x_end = None
        elif (last_x_end is not None and at_x - last_x_end > 0.8 * size and out and not out[-1].endswith(" ")
              and not txt.startswith(" ")):
            out.append(" ")
        out.append(txt)
        line_y = at_y
        last_x_end = at_x + 0.5 * size * len(txt)

    while True:
        try:
            o = ps.obj()
        except (EOFError, IndexError, ValueError):
            break
        if isinstance(o, Op):
            op = o.decode("latin-1")
            if op == "Tf" and len(ops) >= 2:
                font = fonts.get(str(ops[-2]))
                size = abs(float(ops[-1])) if isinstance(ops[-1], (int, float)) else size
            elif op in ("Td", "TD") and len(ops) >= 2:
                x += float(ops[-2])
                y += float(ops[-1])
            elif op == "Tm" and len(ops) >= 6:
                x, y = float(ops[-2]), float(ops[-1])
            elif op == "T*":
                y -= size
            elif op == "BT":
                x = y = 0.0
            elif op in ("Tj", "'", '"') and ops:
                if op != "Tj":
                    y -= size
                s = ops[-1]
                if isinstance(s, bytes):
                    emit(font.decode(s) if font else s.decode("latin-1"), x, y)
            elif op == "TJ" and ops and isinstance(ops[-1], list):
                buf = []
                for el in ops[-1]:
                    if isinstance(el, bytes):
                        buf.append(font.decode(el) if font else el.decode("latin-1"))
                    elif isinstance(el, (int, float)) and el < -200:
                        buf.append(" ")
                emit("".join(buf), x, y)
            elif op == "ET":
                pass
            ops = []
        else:
            ops.append(o)
    text = "".join(out)
    text = re.sub(r"[ \t]+\n", "\n", text)
    return re.sub(r" {2,}", " ", text).strip()


def extract_text(data: bytes) -> List[str]:
    """Text of every page, in page order."""
    doc = PDFDocument(data)
    return [_page_text(doc, p) for p in doc.pages()]


def extract_file(path: str) -> Dict[str, Any]:
    """The reference tool's result shape: {filename, total_pages, content{page_N: text}}."""
    import os

    with open(path, "rb") as f:
        pages = extract_text(f.read())
    return {"filename": os.path.basename(path), "total_pages": len(pages),
            "content": {f"page_{i + 1}": t for i, t in enumerate(pages) if t.strip()}}


# --------------------------------------------------------------------------- writer


def write_simple_pdf(path: str, pages: List[str], compress: bool = True) -> None:
    """Write a minimal valid PDF (Helvetica, one text line per input line)."""
    objs: List[bytes] = []

    def esc(s: str) -> bytes:
        return s.encode("latin-1", "replace").replace(b"\\", b"\\\\").replace(b"(", b"\\(").replace(b")", b"\\)")

    n_pages = len(pages)
    # 1 catalog, 2 pages, 3 font, then (page, content) pairs
    kids = " ".join(f"{4 + 2 * i} 0 R" for i in range(n_pages))
    objs.append(b"<< /Type /Catalog /Pages 2 0 R >>")
    objs.append(f"<< /Type /Pages /Kids [{kids}] /Count {n_pages} >>".encode())
    objs.append(b"<< /Type /Font /Subtype /Type1 /BaseFont /Helvetica /Encoding /WinAnsiEncoding >>")
    for i, text in enumerate(pages):
        lines = text.split("\n")
        body = b"BT /F1 12 Tf 72 760 Td 14 TL\n" + b"".join(b"(" + esc(ln) + b") Tj T*\n" for ln in lines) + b"ET"
        objs.append(f"<< /Type /Page /Parent 2 0 R /MediaBox [0 0 612 792] /Resources << /Font << /F1 3 0 R >> >> "
                    f"/Contents {5 + 2 * i} 0 R >>".encode())
        data = zlib.compress(body) if compress else body
        filt = b" /Filter /FlateDecode" if compress else b""
        objs.append(b"<< /Length " + str(len(data)).encode() + filt + b" >>\nstream\n" + data + b"\nendstream")
    out = bytearray(b"%PDF-1.4\n%\xe2\xe3\xcf\xd3\n")
    offs = []
    for i, o in enumerate(objs):
        offs.append(len(out))
        out += f"{i + 1} 0 obj\n".encode() + o + b"\nendobj\n"
    xref = len(out)
    out += f"xref\n0 {len(objs) + 1}\n0000000000 65535 f \n".encode()
    for off in offs:
        out += f"{off:010d} 00000 n \n".encode()
    out += f"trailer\n<< /Size {len(objs) + 1} /Root 1 0 R >>\nstartxref\n{xref}\n%%EOF\n".encode()
    with open(path, "wb") as f:
        f.write(bytes(out))
