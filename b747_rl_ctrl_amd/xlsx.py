"""Storage.save's workbook without openpyxl: a minimal Office Open XML writer.

The reference's `write_dataframe` (tools/general.py:230-312) writes the Storage table through pandas/openpyxl into
sheet "data" -- the index column (the `base` column, e.g. "t, [с]", or 0..n-1) followed by one column per signal,
labels carrying their units -- and adds one scatter chart per group of columns (the part of the label before the
model separator; "vartheta, [град]" also plots "vartheta_ref, [град]", "h, [м]" / "y, [м]" plot "hzh, [м]"),
anchored at A5, with smoothed lines in the reference's colour x dash-style cycle, Times New Roman axis and legend
text, minor gridlines, arrow-ended axes, the legend at the bottom and series titled by `get_label_desc`.
`bigMode` (the "<stem>_big.xlsx" copy) scales the fonts (14 -> 40 pt) and the line widths (2 -> 7 pt).
`write_frame` is `DataFrame.to_excel(filename)` for the plain tables (ControllerAgent.test's info sheets).
openpyxl is not installed in this image, so the same parts are written here directly with zipfile: the
workbook, sheet "data" (numbers as numeric cells, labels as inline strings, NaN as empty cells like pandas'
na_rep), one drawing and its charts.
"""
import math
import time
import zipfile
from typing import Dict, List, Optional, Sequence
from xml.sax.saxutils import escape

MODEL_SEPARATOR = "__"
LINE_COLORS = ["ff0000", "ff00d5", "4000ff", "00fbff", "7f18c4", "00ff37", "e6ff00", "ff7b00", "707070", "e875ff",
               "ffc875", "ffa6a6", "000000", "4a3d29", "695c0e", "100a38", "7d1d02", "064720"]   # general.py:146-165
LINE_DASH_STYLES = [None, "sysDot"]                                                              # general.py:167-170
EMU_PER_PIXEL = 9525
CHART_CX, CHART_CY = 5400000, 2700000          # openpyxl's default chart size, 15 x 7.5 cm

NS_MAIN = "http://schemas.openxmlformats.org/spreadsheetml/2006/main"
NS_R = "http://schemas.openxmlformats.org/officeDocument/2006/relationships"
NS_PKG = "http://schemas.openxmlformats.org/package/2006/relationships"
NS_C = "http://schemas.openxmlformats.org/drawingml/2006/chart"
NS_A = "http://schemas.openxmlformats.org/drawingml/2006/main"
NS_XDR = "http://schemas.openxmlformats.org/drawingml/2006/spreadsheetDrawing"
REL_DOC = "http://schemas.openxmlformats.org/officeDocument/2006/relationships"
REL_PKG = "http://schemas.openxmlformats.org/package/2006/relationships"
NS_DOC = "http://schemas.openxmlformats.org/officeDocument/2006"


def col_letter(j: int) -> str:
    """0-based column index -> "A", "B", ..., "AA" ..."""
    s = ""
    j += 1
    while j:
        j, r = divmod(j - 1, 26)
        s = chr(65 + r) + s
    return s


def _comp_begin(label: str, target: str) -> bool:
    return len(label) >= len(target) and label[:len(target)] == target


def get_model_name_desc(model_name: str) -> str:
    """tools/general.py:183-215"""
    description = ""
    mapping = {"obs": {"SPEED_MODE": "ПСР", "PID_SPEED_AERO": "ПСРА", "PID_LIKE": "Подобие"},
               "ctrl_mode": {"ADD_DIRECT_CONTROL": "ПКД", "ADD_PROC_CONTROL": "ОКД", "DIRECT_CONTROL": "ПУ"},
               "reset_ref_modes": {"CONST": "ПТУ", "OSCILLATING": "ОЗУ", "HYBRID": "ГИ"},
               "disturbance": {"AERO_DISTURBANCE": "Погрешность а/д"}}
    for m in mapping.values():
        for name, desc in m.items():
            if name in model_name:
                description += " + " + desc if description else desc
                model_name = model_name.replace(name, "")
                break
    return description or model_name.split(MODEL_SEPARATOR)[-1]


def get_label_desc(label: str, index: Optional[int] = None) -> str:
    """tools/general.py:218-227"""
    if _comp_begin(label, "vartheta_ref"):
        return "Требуемый угол тангажа"
    if _comp_begin(label, "hzh"):
        return "Требуемая высота полета"
    if MODEL_SEPARATOR not in label:
        return "СС ПИД"
    if index is not None:
        return f"Конфигурация {index}"
    return get_model_name_desc(label)


def chart_groups(columns: Sequence[str]) -> List[List[str]]:
    """write_dataframe's grouping (tools/general.py:289-303)"""
    groups: Dict[str, List[str]] = {}
    for c in columns:
        groups.setdefault(c.split(MODEL_SEPARATOR)[0] if MODEL_SEPARATOR in c else c, []).append(c)
    out = []
    for labels in groups.values():
        labels = list(labels)
        if labels[0] == "vartheta, [град]":
            labels.append("vartheta_ref, [град]")
        elif labels[0] in ("h, [м]", "y, [м]"):
            labels.append("hzh, [м]")
        out.append(labels)
    return out


def _num(v) -> Optional[str]:
    try:
        f = float(v)
    except (TypeError, ValueError):
        return None
    if math.isnan(f) or math.isinf(f):
        return None
    return repr(f)


def _cell(ref: str, v) -> str:
    n = _num(v)
    if n is not None:
        return f'<c r="{ref}"><v>{n}</v></c>'
    if v is None or (isinstance(v, float) and math.isnan(v)):
        return ""
    return f'<c r="{ref}" t="inlineStr"><is><t>{escape(str(v))}</t></is></c>'


def _sheet_xml(index_name: str, index: Sequence, columns: Sequence[str], data: Sequence[Sequence],
               drawing: bool = True) -> str:
    rows = [f'<row r="1">{_cell("A1", index_name) if index_name else ""}' +
            "".join(_cell(f"{col_letter(j + 1)}1", c) for j, c in enumerate(columns)) + "</row>"]
    for i, iv in enumerate(index):
        r = i + 2
        rows.append(f'<row r="{r}">{_cell(f"A{r}", iv)}' +
                    "".join(_cell(f"{col_letter(j + 1)}{r}", data[j][i]) for j in range(len(columns))) + "</row>")
    draw = '<drawing r:id="rId1"/>' if drawing else ""
    return (f'<?xml version="1.0" encoding="UTF-8" standalone="yes"?>\n<worksheet xmlns="{NS_MAIN}" xmlns:r="{NS_R}">'
            f'<sheetData>{"".join(rows)}</sheetData>{draw}</worksheet>')


def _rich(size: int) -> str:
    cp = f'<a:defRPr sz="{size}" b="0"><a:latin typeface="Times New Roman"/></a:defRPr>'
    return (f'<c:txPr><a:bodyPr/><a:p><a:pPr>{cp}</a:pPr><a:endParaRPr lang="ru-RU" sz="{size}" b="0">'
            f'<a:latin typeface="Times New Roman"/></a:endParaRPr></a:p></c:txPr>')


def _axis(ax_id: int, cross: int, pos: str, title: str, size: int, width: int) -> str:
    t = ""
    if title:
        t = (f'<c:title><c:tx><c:rich><a:bodyPr/><a:p><a:r><a:rPr lang="ru-RU" sz="{size}" b="0">'
             f'<a:latin typeface="Times New Roman"/></a:rPr><a:t>{escape(title)}</a:t></a:r></a:p></c:rich></c:tx>'
             f'<c:overlay val="0"/></c:title>')
    ln = (f'<c:spPr><a:ln w="{width}"><a:solidFill><a:srgbClr val="000000"/></a:solidFill>'
          f'<a:tailEnd type="arrow" len="med"/></a:ln></c:spPr>')
    return (f'<c:valAx><c:axId val="{ax_id}"/><c:scaling><c:orientation val="minMax"/></c:scaling>'
            f'<c:delete val="0"/><c:axPos val="{pos}"/><c:minorGridlines/>{t}<c:numFmt formatCode="General" '
            f'sourceLinked="1"/><c:majorTickMark val="out"/><c:minorTickMark val="none"/><c:tickLblPos val="nextTo"/>'
            f'{ln}{_rich(size)}<c:crossAx val="{cross}"/><c:crosses val="autoZero"/><c:crossBetween val="midCat"/>'
            f'</c:valAx>')


def _chart_xml(labels: Sequence[str], columns: Sequence[str], index_name: str, n_rows: int, big: bool) -> str:
    size = 4000 if big else 1400
    width = round((7 if big else 2) * 96 / 72) * EMU_PER_PIXEL           # points_to_pixels -> pixels_to_EMU
    styles = [(c, d) for c in LINE_COLORS for d in LINE_DASH_STYLES]
    sers = []
    x_ref = f"'data'!$A$2:$A${n_rows + 1}"
    for i, label in enumerate(labels):
        color, dash = styles[i]
        col = col_letter(list(columns).index(label) + 1)
        dash_xml = f'<a:prstDash val="{dash}"/>' if dash else ""
        sers.append(f'<c:ser><c:idx val="{i}"/><c:order val="{i}"/><c:tx><c:v>{escape(get_label_desc(label, i + 1))}'
                    f'</c:v></c:tx><c:spPr><a:ln w="{width}"><a:solidFill><a:srgbClr val="{color}"/></a:solidFill>'
                    f'{dash_xml}</a:ln></c:spPr><c:xVal><c:numRef><c:f>{x_ref}</c:f></c:numRef></c:xVal>'
                    f"<c:yVal><c:numRef><c:f>'data'!${col}$2:${col}${n_rows + 1}</c:f></c:numRef></c:yVal>"
                    f'<c:smooth val="1"/></c:ser>')
    name = labels[0]
    y_title = name.split(MODEL_SEPARATOR)[0] if MODEL_SEPARATOR in name else name
    return (f'<?xml version="1.0" encoding="UTF-8" standalone="yes"?>\n<c:chartSpace xmlns:c="{NS_C}" '
            f'xmlns:a="{NS_A}" xmlns:r="{NS_R}"><c:chart><c:autoTitleDeleted val="1"/><c:plotArea><c:layout/>'
            f'<c:scatterChart><c:scatterStyle val="lineMarker"/><c:varyColors val="0"/>{"".join(sers)}'
            f'<c:axId val="10"/><c:axId val="20"/></c:scatterChart>'
            f'{_axis(10, 20, "b", index_name, size, width)}{_axis(20, 10, "l", y_title, size, width)}</c:plotArea>'
            f'<c:legend><c:legendPos val="b"/><c:overlay val="0"/>{_rich(size)}</c:legend>'
            f'<c:plotVisOnly val="1"/><c:dispBlanksAs val="gap"/></c:chart></c:chartSpace>')


def _drawing_xml(n_charts: int) -> str:
    anchors = []
    for k in range(n_charts):                            # every chart at A5, as ws.add_chart(chart, "A5")
        anchors.append(f'<xdr:oneCellAnchor><xdr:from><xdr:col>0</xdr:col><xdr:colOff>0</xdr:colOff><xdr:row>4'
                       f'</xdr:row><xdr:rowOff>0</xdr:rowOff></xdr:from><xdr:ext cx="{CHART_CX}" cy="{CHART_CY}"/>'
                       f'<xdr:graphicFrame macro=""><xdr:nvGraphicFramePr><xdr:cNvPr id="{k + 1}" name="Chart {k + 1}"/>'
                       f'<xdr:cNvGraphicFramePr/></xdr:nvGraphicFramePr><xdr:xfrm/><a:graphic><a:graphicData '
                       f'uri="{NS_C}"><c:chart xmlns:c="{NS_C}" r:id="rId{k + 1}"/></a:graphicData></a:graphic>'
                       f'</xdr:graphicFrame><xdr:clientData/></xdr:oneCellAnchor>')
    return (f'<?xml version="1.0" encoding="UTF-8" standalone="yes"?>\n<xdr:wsDr xmlns:xdr="{NS_XDR}" '
            f'xmlns:a="{NS_A}" xmlns:r="{NS_R}">{"".join(anchors)}</xdr:wsDr>')


def _rels(items, full=()) -> str:
    """relationships of officeDocument types (items: id, type name, target) and of full type URIs (full)"""
    rel = [(i, f"{REL_DOC}/{t}", tg) for i, t, tg in items] + list(full)
    return (f'<?xml version="1.0" encoding="UTF-8" standalone="yes"?>\n<Relationships xmlns="{NS_PKG}">' +
            "".join(f'<Relationship Id="{i}" Type="{t}" Target="{tg}"/>' for i, t, tg in rel) +
            "</Relationships>")


# The stylesheet every SpreadsheetML consumer may require (one font, the two mandatory fills, one border, the
# "Normal" cell style): cells carry no s= attribute, so all of them use cellXfs 0.
STYLES_XML = ('<?xml version="1.0" encoding="UTF-8" standalone="yes"?>\n'
              '<styleSheet xmlns="http://schemas.openxmlformats.org/spreadsheetml/2006/main">'
              '<fonts count="1"><font><sz val="11"/><name val="Calibri"/><family val="2"/></font></fonts>'
              '<fills count="2"><fill><patternFill patternType="none"/></fill>'
              '<fill><patternFill patternType="gray125"/></fill></fills>'
              '<borders count="1"><border><left/><right/><top/><bottom/><diagonal/></border></borders>'
              '<cellStyleXfs count="1"><xf numFmtId="0" fontId="0" fillId="0" borderId="0"/></cellStyleXfs>'
              '<cellXfs count="1"><xf numFmtId="0" fontId="0" fillId="0" borderId="0" xfId="0"/></cellXfs>'
              '<cellStyles count="1"><cellStyle name="Normal" xfId="0" builtinId="0"/></cellStyles>'
              '</styleSheet>')


def _core_xml() -> str:
    now = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
    return ('<?xml version="1.0" encoding="UTF-8" standalone="yes"?>\n<cp:coreProperties '
            'xmlns:cp="http://schemas.openxmlformats.org/package/2006/metadata/core-properties" '
            'xmlns:dc="http://purl.org/dc/elements/1.1/" xmlns:dcterms="http://purl.org/dc/terms/" '
            'xmlns:xsi="http://www.w3.org/2001/XMLSchema-instance"><dc:creator>b747_rl_ctrl_amd</dc:creator>'
            f'<dcterms:created xsi:type="dcterms:W3CDTF">{now}</dcterms:created>'
            f'<dcterms:modified xsi:type="dcterms:W3CDTF">{now}</dcterms:modified></cp:coreProperties>')


def write_table(filename: str, index_name: str, index: Sequence, columns: Sequence[str], data: Sequence[Sequence],
                big: bool = False, charts: bool = True, sheet: str = "data") -> str:
    """write_dataframe(data, filename, bigMode=big): sheet "data" (index column + columns) and its charts;
    charts=False, sheet="Sheet1": a plain DataFrame.to_excel(filename) table"""
    groups = [[c for c in g if c in columns] for g in chart_groups(columns)] if charts else []
    n = len(index)
    ct = ['<Default Extension="rels" ContentType="application/vnd.openxmlformats-package.relationships+xml"/>',
          '<Default Extension="xml" ContentType="application/xml"/>',
          '<Override PartName="/xl/workbook.xml" '
          'ContentType="application/vnd.openxmlformats-officedocument.spreadsheetml.sheet.main+xml"/>',
          '<Override PartName="/xl/worksheets/sheet1.xml" '
          'ContentType="application/vnd.openxmlformats-officedocument.spreadsheetml.worksheet+xml"/>']
    if groups:
        ct.append('<Override PartName="/xl/drawings/drawing1.xml" '
                  'ContentType="application/vnd.openxmlformats-officedocument.drawing+xml"/>')
    ct += [f'<Override PartName="/xl/charts/chart{k + 1}.xml" '
           f'ContentType="application/vnd.openxmlformats-officedocument.drawingml.chart+xml"/>' for k in range(len(groups))]
    ct += ['<Override PartName="/xl/styles.xml" '
           'ContentType="application/vnd.openxmlformats-officedocument.spreadsheetml.styles+xml"/>',
           '<Override PartName="/docProps/core.xml" '
           'ContentType="application/vnd.openxmlformats-package.core-properties+xml"/>',
           '<Override PartName="/docProps/app.xml" '
           'ContentType="application/vnd.openxmlformats-officedocument.extended-properties+xml"/>']
    with zipfile.ZipFile(filename, "w", zipfile.ZIP_DEFLATED) as z:
        z.writestr("[Content_Types].xml", '<?xml version="1.0" encoding="UTF-8" standalone="yes"?>\n<Types xmlns='
                   '"http://schemas.openxmlformats.org/package/2006/content-types">' + "".join(ct) + "</Types>")
        z.writestr("_rels/.rels", _rels([("rId1", "officeDocument", "xl/workbook.xml")],
                                        [("rId2", f"{REL_PKG}/metadata/core-properties", "docProps/core.xml"),
                                         ("rId3", f"{REL_DOC}/extended-properties", "docProps/app.xml")]))
        z.writestr("docProps/core.xml", _core_xml())
        z.writestr("docProps/app.xml", f'<?xml version="1.0" encoding="UTF-8" standalone="yes"?>\n<Properties '
                   f'xmlns="{NS_DOC}/extended-properties"><Application>b747_rl_ctrl_amd</Application></Properties>')
        z.writestr("xl/workbook.xml", f'<?xml version="1.0" encoding="UTF-8" standalone="yes"?>\n<workbook '
                   f'xmlns="{NS_MAIN}" xmlns:r="{NS_R}"><sheets><sheet name="{escape(sheet)}" sheetId="1" '
                   f'r:id="rId1"/></sheets></workbook>')
        z.writestr("xl/_rels/workbook.xml.rels", _rels([("rId1", "worksheet", "worksheets/sheet1.xml"),
                                                        ("rId2", "styles", "styles.xml")]))
        z.writestr("xl/styles.xml", STYLES_XML)
        z.writestr("xl/worksheets/sheet1.xml", _sheet_xml(index_name, index, columns, data, bool(groups)))
        if not groups:
            return filename
        z.writestr("xl/worksheets/_rels/sheet1.xml.rels", _rels([("rId1", "drawing", "../drawings/drawing1.xml")]))
        z.writestr("xl/drawings/drawing1.xml", _drawing_xml(len(groups)))
        z.writestr("xl/drawings/_rels/drawing1.xml.rels",
                   _rels([(f"rId{k + 1}", "chart", f"../charts/chart{k + 1}.xml") for k in range(len(groups))]))
        for k, g in enumerate(groups):
            z.writestr(f"xl/charts/chart{k + 1}.xml", _chart_xml(g, columns, index_name, n, big))
    return filename


def write_frame(filename: str, df) -> str:
    """DataFrame.to_excel(filename, index=True, header=True): sheet "Sheet1", the index then the columns"""
    return write_table(filename, "" if df.index.name is None else str(df.index.name), df.index.tolist(),
                       [str(c) for c in df.columns], [df[c].tolist() for c in df.columns], charts=False,
                       sheet="Sheet1")
