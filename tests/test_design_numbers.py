"""Every number in DESIGN.md's "Measured numbers" table matches the profile it cites (round-4
review item 4: DESIGN.md is a current-state document whose numbers are the latest profiles').

The table's rows are `| quantity | value | file | key |`:
- `file` is a path under the repo (a committed profile);
- `key` selects the number in it:
  - `.json`: a dotted path (`roofline.frac`; list indices as numbers);
  - `.jsonl`: `field=value,field=value|path`: the first row whose fields equal those values (as
    strings), then the dotted path in it;
  - `.csv`: `column=substring|column`: the first row whose column contains the substring;
  - a trailing `*factor` scales the file's number (e.g. ns -> µs: `*0.001`).
- `value` is the number as DESIGN.md prints it (thin spaces and thousands separators allowed); the
  file's number, scaled, must round to it at the printed precision.
"""
import csv
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _table_rows():
    with open(os.path.join(ROOT, "DESIGN.md")) as fh:
        text = fh.read()
    start = text.index("<!-- measured-numbers:begin -->")
    end = text.index("<!-- measured-numbers:end -->")
    rows = []
    for line in text[start:end].splitlines():
        if not line.strip().startswith("|"):
            continue
        # cells split on unescaped pipes; a key's own "|" is written "\|" in the markdown
        cells = [c.strip().replace("\\|", "|") for c in re.split(r"(?<!\\)\|", line.strip().strip("|"))]
        if len(cells) != 4:
            raise ValueError(f"measured-numbers row without 4 cells: {line!r}")
        if cells[0] in ("quantity", "") or set(cells[1]) <= set("-: "):
            continue
        rows.append(tuple(cells))
    return rows


def _path(obj, dotted):
    """A dotted path; a dict key that itself holds dots (``speedup@50GBps,delta0.1``) is matched
    whole before the path is split."""
    if isinstance(obj, dict) and dotted in obj:
        return obj[dotted]
    head, _, rest = dotted.partition(".")
    obj = obj[int(head)] if isinstance(obj, list) else obj[head]
    return _path(obj, rest) if rest else obj


def _lookup(file, key):
    factor = 1.0
    if "*" in key:
        key, f = key.rsplit("*", 1)
        factor = float(f)
    path = os.path.join(ROOT, file.strip("`"))
    if path.endswith(".json"):
        with open(path) as fh:
            return float(_path(json.load(fh), key)) * factor
    if path.endswith(".jsonl"):
        sel, _, dotted = key.partition("|")
        # field=value pairs; a value may hold commas (split only before the next "field=")
        conds = [c.split("=", 1) for c in re.split(r",(?=[A-Za-z_]\w*=)", sel) if c]
        with open(path) as fh:
            for line in fh:
                line = line.strip()
                if not line.startswith("{"):
                    continue
                row = json.loads(line)
                if all(str(row.get(k)) == v for k, v in conds):
                    return float(_path(row, dotted)) * factor
        raise KeyError(f"no row of {file} matches {sel}")
    if path.endswith(".csv"):
        sel, _, col = key.partition("|")
        ccol, sub = sel.split("=", 1)
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if sub in row[ccol]:
                    return float(row[col]) * factor
        raise KeyError(f"no row of {file} has {sub} in {ccol}")
    raise ValueError(f"unsupported profile type {file}")


def _printed(value):
    v = value.replace(" ", "").replace(" ", "").replace(",", "").replace("**", "")
    m = re.match(r"^-?\d+(\.\d+)?", v)
    assert m, value
    num = m.group(0)
    decimals = len(num.split(".")[1]) if "." in num else 0
    return float(num), decimals


try:
    ROWS = _table_rows()
except (OSError, ValueError):  # reported by test_table_is_there_and_cites_only_committed_profiles
    ROWS = []


def test_table_is_there_and_cites_only_committed_profiles():
    assert len(_table_rows()) == len(ROWS) >= 30  # every row parsed (none skipped)
    for _, _, file, _ in ROWS:
        assert os.path.exists(os.path.join(ROOT, file.strip("`"))), file


@pytest.mark.parametrize("quantity,value,file,key", ROWS, ids=[r[0][:40] for r in ROWS])
def test_design_number_matches_its_profile(quantity, value, file, key):
    shown, decimals = _printed(value)
    got = _lookup(file, key.strip("`"))
    assert round(got, decimals) == pytest.approx(shown, abs=0.5 * 10 ** -decimals + 1e-12), \
        f"{quantity}: DESIGN.md says {value}, {file} [{key}] holds {got}"


def test_design_is_a_current_state_document():
    """Under ~50 KB, and the round-by-round notebook lives in docs/history.md."""
    assert os.path.getsize(os.path.join(ROOT, "DESIGN.md")) < 50_000
    assert os.path.exists(os.path.join(ROOT, "docs", "history.md"))
