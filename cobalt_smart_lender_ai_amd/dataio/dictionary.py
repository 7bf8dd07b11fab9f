"""LendingClub data dictionary.

The reference ships ``data/1-raw/lending-club-2007-2020Q3/LCDataDictionary.xlsx`` (column name ->
description) as documentation of the raw CSV's 150+ columns. An ``.xlsx`` file is a zip archive of
XML parts, so it is read here with the standard library only (``zipfile`` + ``xml.etree``): no
spreadsheet engine is needed and nothing in the file is executed.

``load_data_dictionary(path)`` returns ``{column: description}``; ``describe_columns(columns, dd)``
resolves engineered column names (one-hot dummies, ``_NA`` indicators, ``emp_length_num``,
``*_days``) to their source column's description.
"""
from __future__ import annotations

import re
import zipfile
from pathlib import Path
from xml.etree import ElementTree as ET

_M = "http://schemas.openxmlformats.org/spreadsheetml/2006/main"
_R = "http://schemas.openxmlformats.org/officeDocument/2006/relationships"
_PR = "http://schemas.openxmlformats.org/package/2006/relationships"
_NS = {"m": _M}

# where the reference keeps the workbook (relative to its repository root)
REFERENCE_PATH = "data/1-raw/lending-club-2007-2020Q3/LCDataDictionary.xlsx"


def _col_index(ref: str) -> int:
    """'A1' -> 0, 'B7' -> 1, 'AA3' -> 26."""
    idx = 0
    for ch in re.match(r"[A-Z]+", ref).group(0):
        idx = idx * 26 + (ord(ch) - 64)
    return idx - 1


def _text(el) -> str:
    # a shared/inline string is a plain <t> or a list of rich-text runs <r><t>
    return "".join(t.text or "" for t in el.iter(f"{{{_M}}}t"))


def _shared_strings(z: zipfile.ZipFile) -> list[str]:
    try:
        root = ET.fromstring(z.read("xl/sharedStrings.xml"))
    except KeyError:
        return []
    return [_text(si) for si in root.findall("m:si", _NS)]


def _sheet_parts(z: zipfile.ZipFile) -> list[tuple[str, str]]:
    """(sheet name, part path) in workbook order."""
    wb = ET.fromstring(z.read("xl/workbook.xml"))
    rels = ET.fromstring(z.read("xl/_rels/workbook.xml.rels"))
    target = {r.get("Id"): r.get("Target") for r in rels.findall(f"{{{_PR}}}Relationship")}
    out = []
    for s in wb.find("m:sheets", _NS).findall("m:sheet", _NS):
        t = target.get(s.get(f"{{{_R}}}id"), "").lstrip("/")
        out.append((s.get("name"), t if t.startswith("xl/") else "xl/" + t))
    return out


def sheet_names(path: str | Path) -> list[str]:
    with zipfile.ZipFile(path) as z:
        return [n for n, _ in _sheet_parts(z)]


def read_xlsx_rows(path: str | Path, sheet: int | str = 0) -> list[list[str]]:
    """All non-empty rows of one worksheet as lists of strings (missing cells -> '')."""
    with zipfile.ZipFile(path) as z:
        strings = _shared_strings(z)
        parts = _sheet_parts(z)
        part = dict(parts)[sheet] if isinstance(sheet, str) else parts[sheet][1]
        root = ET.fromstring(z.read(part))
    rows: list[list[str]] = []
    for row in root.iter(f"{{{_M}}}row"):
        cells: dict[int, str] = {}
        for c in row.findall("m:c", _NS):
            kind, v = c.get("t"), c.find("m:v", _NS)
            if kind == "s" and v is not None:
                val = strings[int(v.text)]
            elif kind == "inlineStr":
                val = _text(c)
            else:
                val = v.text if v is not None and v.text is not None else ""
            ref = c.get("r")
            cells[_col_index(ref) if ref else len(cells)] = val
        if any(x.strip() for x in cells.values()):
            rows.append([cells.get(i, "") for i in range(max(cells) + 1)])
    return rows


def load_data_dictionary(path: str | Path, sheet: int | str = 0) -> dict[str, str]:
    """``{column name: description}`` from the LendingClub workbook (first sheet, header
    ``LoanStatNew`` / ``Description``). Names are stripped; rows without a name are skipped."""
    rows = read_xlsx_rows(path, sheet)
    if not rows:
        return {}
    header = [h.strip().lower() for h in rows[0]]
    name_col = next((i for i, h in enumerate(header) if h in ("loanstatnew", "browsenotesfile", "name")), 0)
    desc_col = next((i for i, h in enumerate(header) if h == "description"), 1)
    out: dict[str, str] = {}
    for r in rows[1:]:
        if len(r) <= name_col:
            continue
        name = r[name_col].strip()
        if name:
            out[name] = r[desc_col].strip() if desc_col < len(r) else ""
    return out


def source_column(column: str, known) -> str:
    """The raw column an engineered column comes from (``grade_E`` -> ``grade``,
    ``emp_length_num`` -> ``emp_length``, ``dti_NA`` -> ``dti``, ``earliest_cr_line_days`` ->
    ``earliest_cr_line``); the name itself when it is already known or cannot be resolved."""
    low = {k.lower() for k in known}
    if column.lower() in low:
        return column
    base = column
    for suffix in ("_NA", "_num", "_days"):
        if base.endswith(suffix) and base[: -len(suffix)].lower() in low:
            return base[: -len(suffix)]
    head = base
    while "_" in head:  # one-hot dummies: strip the level (which may contain '_' or spaces)
        head = head.rsplit("_", 1)[0]
        if head.lower() in low:
            return head
    return column


def describe_columns(columns, dd: dict[str, str]) -> dict[str, str]:
    """Description of every column ('' when the dictionary has no entry for its source column)."""
    lower = {k.lower(): v for k, v in dd.items()}
    return {c: lower.get(source_column(c, dd).lower(), "") for c in columns}
