"""The SharedStrings behind the reference's summary fixtures, rebuilt.

packages/dds/sequence/src/test/generateSharedStrings.ts:47-147 builds each
fixture's string from local edits on a fresh SharedString (no collaboration:
every segment is NonCollabClient at UniversalSequenceNumber) and
createSnapshotFiles.ts summarizes it.  strings(name) replays those edits on a
plain segment list — insertText splits at the position and adds a segment,
insertMarker adds a marker, annotateRange splits at both ends and sets props —
and returns the segments in order as the interned specs load_bodies takes,
plus the text / per-position props the loaded document must read."""
from fluidframework_amd.packing import Interner, utf16_units

SIZE_OF_FIRST_CHUNK = 10000  # SnapshotLegacy.sizeOfFirstChunk
INSERT_TEXT = "text"
MARKER_PROPS = lambda i: {"ItemType": "Paragraph", "Properties": {"Bold": False},  # noqa: E731
                          "markerId": f"marker{i}", "referenceTileLabels": ["Eop"]}
TILE = 1  # ReferenceType.Tile


class SegList:
    def __init__(self):
        self.segs = []  # [text | None (marker), props dict, refType]

    def length(self):
        return sum(len(s[0]) if s[0] is not None else 1 for s in self.segs)

    def _split(self, pos):
        """Index of the first segment starting at pos (splitting one that spans it)."""
        p = 0
        for i, s in enumerate(self.segs):
            n = len(s[0]) if s[0] is not None else 1
            if p == pos:
                return i
            if p < pos < p + n:
                self.segs[i:i + 1] = [[s[0][:pos - p], dict(s[1]), s[2]], [s[0][pos - p:], dict(s[1]), s[2]]]
                return i + 1
            p += n
        return len(self.segs)

    def insert_text(self, pos, text):
        self.segs.insert(self._split(pos), [text, {}, 0])

    def insert_marker(self, pos, ref_type, props):
        self.segs.insert(self._split(pos), [None, dict(props), ref_type])

    def annotate(self, start, end, props):
        a = self._split(start)
        b = self._split(end)
        for s in self.segs[a:b]:
            s[1].update(props)


def build(name):
    """generateSharedStrings.ts:70-130 for one fixture name (the version prefix does
    not change the content)."""
    kind = name.split("/")[-1]
    s = SegList()
    if kind in ("headerOnly", "withIntervals", "withV1Intervals"):
        for i in range(SIZE_OF_FIRST_CHUNK // len(INSERT_TEXT) // 2):
            s.insert_text(0, f"{INSERT_TEXT}{i}")
    elif kind == "largeBody":
        for i in range(SIZE_OF_FIRST_CHUNK):
            s.insert_text(0, f"{INSERT_TEXT}-{i}")
    else:
        for i in range(SIZE_OF_FIRST_CHUNK // len(INSERT_TEXT) * 2):
            s.insert_text(0, f"{INSERT_TEXT}{i}")
        if kind == "withMarkers":
            i = 0
            while i < s.length():
                s.insert_marker(i, TILE, MARKER_PROPS(i))
                i += 70
        elif kind == "withAnnotations":
            for i in range(0, s.length(), 70):
                s.annotate(i, i + 10, {"bold": True})
    return s


def body(seglist, interner):
    """-> [{"json": interned spec}] for load_bodies (seq 0 / no client: below the MSN)."""
    out = []
    for text, props, ref_type in seglist.segs:
        p = {interner.key(k): interner.value(v) for k, v in props.items()}
        if text is None:
            j = {"marker": {"refType": ref_type}}
        elif p:
            j = {"text": utf16_units(text).tolist()}
        else:
            j = utf16_units(text).tolist()
        if p:
            j["props"] = p
        out.append({"json": j})
    return out


def expected_view(seglist):
    """(text as getText reads it: markers contribute nothing, per-position props)."""
    text, props = [], []
    for t, p, _ in seglist.segs:
        if t is None:
            props.append(dict(p))
        else:
            text.append(t)
            props.extend(dict(p) for _ in t)
    return "".join(text), props


NAMES = ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations", "withIntervals"]


def interner():
    return Interner(8)
