"""LendingClub data dictionary reader: standard-library xlsx parsing."""
import zipfile
from pathlib import Path

import pytest

from cobalt_smart_lender_ai_amd import cli
from cobalt_smart_lender_ai_amd.dataio import dictionary as dd
from cobalt_smart_lender_ai_amd.dataio import synth

REF_XLSX = Path("/root/reference") / dd.REFERENCE_PATH


def _col(i: int) -> str:
    s = ""
    i += 1
    while i:
        i, r = divmod(i - 1, 26)
        s = chr(65 + r) + s
    return s


def _write_xlsx(path, rows):
    """A minimal workbook: text cells as shared strings (one as an inline string), numbers as values."""
    strings, index, xml_rows = [], {}, []
    for ri, row in enumerate(rows, 1):
        cells = []
        for ci, v in enumerate(row):
            ref = f"{_col(ci)}{ri}"
            if v is None:
                continue
            if isinstance(v, str) and v.startswith("inline:"):
                cells.append(f'<c r="{ref}" t="inlineStr"><is><t>{v[7:]}</t></is></c>')
            elif isinstance(v, str):
                index.setdefault(v, len(strings))
                if index[v] == len(strings):
                    strings.append(v)
                cells.append(f'<c r="{ref}" t="s"><v>{index[v]}</v></c>')
            else:
                cells.append(f'<c r="{ref}"><v>{v}</v></c>')
        xml_rows.append(f'<row r="{ri}">{"".join(cells)}</row>')
    m = 'xmlns="http://schemas.openxmlformats.org/spreadsheetml/2006/main"'
    r = 'xmlns:r="http://schemas.openxmlformats.org/officeDocument/2006/relationships"'
    rel = "http://schemas.openxmlformats.org/officeDocument/2006/relationships/worksheet"
    with zipfile.ZipFile(path, "w") as z:
        z.writestr("xl/workbook.xml", f'<workbook {m} {r}><sheets><sheet name="LoanStats" sheetId="1" r:id="rId1"/>'
                                      f'</sheets></workbook>')
        z.writestr("xl/_rels/workbook.xml.rels",
                   '<Relationships xmlns="http://schemas.openxmlformats.org/package/2006/relationships">'
                   f'<Relationship Id="rId1" Type="{rel}" Target="worksheets/sheet1.xml"/></Relationships>')
        z.writestr("xl/worksheets/sheet1.xml", f'<worksheet {m}><sheetData>{"".join(xml_rows)}</sheetData></worksheet>')
        z.writestr("xl/sharedStrings.xml",
                   f"<sst {m}>" + "".join(f"<si><t>{s}</t></si>" for s in strings) + "</sst>")


def test_reader_on_synthetic_workbook(tmp_path):
    p = tmp_path / "dd.xlsx"
    _write_xlsx(p, [["LoanStatNew", "Description"], ["loan_amnt", "The listed amount of the loan"],
                    ["grade", "LC assigned loan grade"], [None, "orphan"], ["term", "inline:Number of payments"],
                    ["int_rate", 7], ["emp_length", "Employment length in years"], ["dti", "Debt to income"]])
    assert dd.sheet_names(p) == ["LoanStats"]
    d = dd.load_data_dictionary(p)
    assert d == {"loan_amnt": "The listed amount of the loan", "grade": "LC assigned loan grade",
                 "term": "Number of payments", "int_rate": "7", "emp_length": "Employment length in years",
                 "dti": "Debt to income"}
    desc = dd.describe_columns(["grade_E", "loan_amnt", "emp_length_num", "dti_NA", "hardship_status_No Hardship"], d)
    assert desc == {"grade_E": "LC assigned loan grade", "loan_amnt": "The listed amount of the loan",
                    "emp_length_num": "Employment length in years", "dti_NA": "Debt to income",
                    "hardship_status_No Hardship": ""}


@pytest.mark.skipif(not REF_XLSX.exists(), reason="reference data dictionary not mounted")
def test_reference_dictionary_covers_the_deployed_features(capsys):
    d = dd.load_data_dictionary(REF_XLSX)
    assert len(d) > 140
    assert d["loan_amnt"].startswith("The listed amount of the loan")
    desc = dd.describe_columns(synth.FEATURES, d)
    assert all(desc[c] for c in synth.FEATURES)  # every deployed feature resolves to a documented column
    assert desc["hardship_status_No Hardship"] == d["hardship_status"]
    assert desc["earliest_cr_line_days"] == d["earliest_cr_line"]
    assert cli.main(["dictionary", "--xlsx", str(REF_XLSX), "grade_E"]) == 0
    assert capsys.readouterr().out.startswith("grade_E\tLC assigned loan grade")
