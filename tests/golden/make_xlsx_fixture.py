"""Package structure of the reference's own openpyxl-written workbook (tensorboard.xlsx: write_dataframe's output,
tools/general.py:230-312) -> tests/golden/xlsx_package.json: the content type of each part kind and the
relationship types of the package and the workbook.  Data only (no cell values).  Run once in the build container:
python tests/golden/make_xlsx_fixture.py /root/reference/tensorboard.xlsx"""
import json
import os
import re
import sys
import zipfile
import xml.etree.ElementTree as ET


def kind(part):
    return re.sub(r"\d+(?=\.xml$)", "N", part.lstrip("/"))


def structure(path):
    with zipfile.ZipFile(path) as z:
        ct = ET.fromstring(z.read("[Content_Types].xml"))
        over = {kind(e.get("PartName")): e.get("ContentType") for e in ct if e.tag.endswith("Override")}
        rels = {}
        for r in ("_rels/.rels", "xl/_rels/workbook.xml.rels", "xl/worksheets/_rels/sheet1.xml.rels"):
            if r in z.namelist():
                rels[r] = sorted(e.get("Type") for e in ET.fromstring(z.read(r)))
        sheet = ET.fromstring(z.read("xl/workbook.xml")).find(
            "{http://schemas.openxmlformats.org/spreadsheetml/2006/main}sheets")[0].get("name")
        return {"parts": sorted({kind(n) for n in z.namelist()}), "content_types": over, "rels": rels,
                "sheet": sheet}


if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "xlsx_package.json")
    json.dump(structure(sys.argv[1]), open(out, "w"), indent=1, sort_keys=True)
    print(out)
