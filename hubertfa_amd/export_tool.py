"""Output writers (reference: tools/export_tool.py:7-92).

* ``<wav_dir>/TextGrid/<stem>.TextGrid`` (or ``<out_path>/TextGrid/``) with IntervalTiers ``words`` and ``phones``
  in Praat long-text format, laid out like the ``textgrid`` PyPI package's ``TextGrid.write`` (gaps filled with
  empty intervals, xmax = last interval end).  The ``textgrid`` package is absent here, so byte-level parity with
  it is UNPINNED; the format is Praat's ooTextFile and is read back by tests/test_host.py.
* ``<wav_dir>/confidence/confidence.csv`` with columns ``name,confidence`` (pandas ``to_csv``, as the reference).
"""
from __future__ import annotations

import pathlib


class _Interval:
    __slots__ = ("minTime", "maxTime", "mark")

    def __init__(self, minTime, maxTime, mark):
        if minTime >= maxTime:   # Praat has no zero/negative-length intervals
            raise ValueError(minTime, maxTime)
        # numpy float64 -> float: the same value and the same text when formatted, without numpy's slow __format__
        minTime = float(minTime) if isinstance(minTime, float) else minTime
        maxTime = float(maxTime) if isinstance(maxTime, float) else maxTime
        self.minTime, self.maxTime, self.mark = minTime, maxTime, mark


class IntervalTier:
    def __init__(self, name=None, minTime=0.0, maxTime=None):
        self.name, self.minTime, self.maxTime = name, minTime, maxTime
        self.intervals: list[_Interval] = []

    def add(self, minTime, maxTime, mark):
        iv = _Interval(minTime, maxTime, mark)
        if iv.minTime < self.minTime:
            raise ValueError(self.minTime)
        if self.maxTime and iv.maxTime > self.maxTime:
            raise ValueError(self.maxTime)
        ivs = self.intervals
        if not ivs or ivs[-1].minTime < iv.minTime:      # in-order adds (the decoder's): O(1), not a linear scan
            pos = len(ivs)
        else:
            pos = 0
            while pos < len(ivs) and ivs[pos].minTime < iv.minTime:
                pos += 1
        for nb in self.intervals[max(pos - 1, 0):pos + 1]:
            if nb.minTime < iv.maxTime and iv.minTime < nb.maxTime:
                raise ValueError("overlapping intervals", nb.minTime, nb.maxTime, minTime, maxTime)
        self.intervals.insert(pos, iv)

    def filled(self, null=""):
        out, prev = [], self.minTime
        for iv in self.intervals:
            if prev < iv.minTime:
                out.append(_Interval(prev, iv.minTime, null))
            out.append(iv)
            prev = iv.maxTime
        if self.maxTime is not None and prev < self.maxTime:
            out.append(_Interval(prev, self.maxTime, null))
        return out


class TextGrid:
    def __init__(self, name=None, minTime=0.0, maxTime=None):
        self.name, self.minTime, self.maxTime = name, minTime, maxTime
        self.tiers: list[IntervalTier] = []

    def append(self, tier):
        if self.maxTime is not None and tier.maxTime is not None and tier.maxTime > self.maxTime:
            raise ValueError(self.maxTime)
        self.tiers.append(tier)

    def lines(self, null=""):
        maxT = self.maxTime or max((t.maxTime if t.maxTime else t.intervals[-1].maxTime) for t in self.tiers)
        yield 'File type = "ooTextFile"'
        yield 'Object class = "TextGrid"'
        yield ""
        yield f"xmin = {self.minTime}"
        yield f"xmax = {maxT}"
        yield "tiers? <exists>"
        yield f"size = {len(self.tiers)}"
        yield "item []:"
        for i, tier in enumerate(self.tiers, 1):
            ivs = tier.filled(null)
            yield f"\titem [{i}]:"
            yield '\t\tclass = "IntervalTier"'
            yield f'\t\tname = "{tier.name}"'
            yield f"\t\txmin = {tier.minTime}"
            yield f"\t\txmax = {maxT}"
            yield f"\t\tintervals: size = {len(ivs)}"
            for j, iv in enumerate(ivs, 1):      # one chunk of four lines per interval
                mark = str(iv.mark).replace('"', '""')
                yield (f'\t\t\tintervals [{j}]:\n\t\t\t\txmin = {iv.minTime}\n\t\t\t\txmax = {iv.maxTime}\n'
                       f'\t\t\t\ttext = "{mark}"')

    def write(self, path, null=""):
        text = "\n".join(self.lines(null)) + "\n"
        with open(path, "w", encoding="utf-8") as f:
            f.write(text)


def read_textgrid(path):
    """Minimal reader of the long text format written above -> {tier: [(xmin, xmax, text), ...]}."""
    tiers, cur, iv = {}, None, {}
    for raw in open(path, encoding="utf-8"):
        s = raw.strip()
        if s.startswith("name = "):
            cur = s[len('name = "'):-1]
            tiers[cur] = []
        elif cur is not None and s.startswith("xmin = ") and raw.startswith("\t\t\t\t"):
            iv = {"xmin": float(s[7:])}
        elif cur is not None and s.startswith("xmax = ") and raw.startswith("\t\t\t\t"):
            iv["xmax"] = float(s[7:])
        elif cur is not None and s.startswith("text = "):
            tiers[cur].append((iv["xmin"], iv["xmax"], s[len('text = "'):-1].replace('""', '"')))
    return tiers


def _tier_rows(seq, intervals, start_as_float, null=""):
    """(start, end, mark) of one tier with its gaps filled by ``null``, the values exactly as IntervalTier.add
    stores them (``start_as_float``: the phones tier's float(start)), for in-order, non-overlapping intervals
    starting at >= 0; None when the tier needs IntervalTier's general path (out of order, overlapping, empty or
    negative-length intervals, which it sorts or rejects, or float32 arrays, whose scalars it keeps as numpy)."""
    if hasattr(intervals, "dtype"):
        if intervals.dtype != "float64":
            return None
        intervals = intervals.tolist()           # numpy f64 -> float: the conversion _Interval applies
    rows, prev = [], 0.0
    for mark, (a, b) in zip(seq, intervals):
        a = float(a) if start_as_float or isinstance(a, float) else a
        b = float(b) if isinstance(b, float) else b
        if not (a < b) or a < prev:
            return None
        if prev < a:
            rows.append((prev, a, null))
        rows.append((a, b, mark))
        prev = b
    return rows


def textgrid_text(word_seq, word_intervals, ph_seq, ph_intervals, null=""):
    """The file ``Exporter`` writes for one prediction (TextGrid with tiers ``words`` and ``phones``), built
    straight from the interval arrays; None when a tier needs the general IntervalTier path."""
    tiers = [("words", _tier_rows(word_seq, word_intervals, False, null)),
             ("phones", _tier_rows(ph_seq, ph_intervals, True, null))]
    if any(r is None or not r for _, r in tiers):
        return None
    maxT = max(r[-1][1] for _, r in tiers)
    out = ['File type = "ooTextFile"', 'Object class = "TextGrid"', "", "xmin = 0.0", f"xmax = {maxT}",
           "tiers? <exists>", f"size = {len(tiers)}", "item []:"]
    for i, (name, rows) in enumerate(tiers, 1):
        out += [f"\titem [{i}]:", '\t\tclass = "IntervalTier"', f'\t\tname = "{name}"', "\t\txmin = 0.0",
                f"\t\txmax = {maxT}", f"\t\tintervals: size = {len(rows)}"]
        # a tier's intervals are contiguous, so each boundary is formatted once: an interval's xmin reuses the
        # previous xmax's text when it is the same value of the same type (zeros are formatted again: -0.0)
        prev, sprev = None, None
        for j, (a, b, m) in enumerate(rows, 1):
            sa = sprev if (a == prev and type(a) is type(prev) and a != 0) else str(a)
            sb = str(b)
            m = str(m)
            if '"' in m:
                m = m.replace('"', '""')
            out.append('\t\t\tintervals [%d]:\n\t\t\t\txmin = %s\n\t\t\t\txmax = %s\n\t\t\t\ttext = "%s"'
                       % (j, sa, sb, m))
            prev, sprev = b, sb
    return "\n".join(out) + "\n"


class Exporter:
    def __init__(self, predictions, log, out_path=None):
        self.predictions = predictions
        self.log = log
        self.out_path = pathlib.Path(out_path) if out_path else None

    def write_textgrid(self, prediction, made=None):
        """One prediction's ``TextGrid/<stem>.TextGrid``; ``made`` caches the folders already created."""
        wav_path, wav_length, confidence, ph_seq, ph_intervals, word_seq, word_intervals = prediction
        wav_path = pathlib.Path(wav_path)
        base = self.out_path if self.out_path is not None else wav_path.parent
        tg_path = base / "TextGrid" / wav_path.with_suffix(".TextGrid").name
        if made is None or tg_path.parent not in made:
            tg_path.parent.mkdir(parents=True, exist_ok=True)
            if made is not None:
                made.add(tg_path.parent)
        text = textgrid_text(word_seq, word_intervals, ph_seq, ph_intervals)
        if text is not None:                 # in-order intervals (post-processing's output): one formatting pass
            with open(tg_path, "w", encoding="utf-8") as f:
                f.write(text)
            return
        tg = TextGrid()
        word_tier = IntervalTier(name="words")
        ph_tier = IntervalTier(name="phones")
        for word, (start, end) in zip(word_seq, word_intervals):
            word_tier.add(start, end, word)
        for ph, (start, end) in zip(ph_seq, ph_intervals):
            ph_tier.add(minTime=float(start), maxTime=end, mark=ph)
        tg.append(word_tier)
        tg.append(ph_tier)
        tg.write(tg_path)

    def save_textgrids(self):
        print("Saving TextGrids...")
        made = set()
        for prediction in self.predictions:
            self.write_textgrid(prediction, made)

    def save_confidence_fn(self):
        import pandas as pd
        print("saving confidence...")
        per_folder = {}
        for wav_path, _, confidence, *_ in self.predictions:
            wav_path = pathlib.Path(wav_path)
            d = per_folder.setdefault(wav_path.parent, {"name": [], "confidence": []})
            d["name"].append(wav_path.with_suffix("").name)
            d["confidence"].append(confidence)
        for folder, data in per_folder.items():
            path = folder / "confidence"
            path.mkdir(parents=True, exist_ok=True)
            pd.DataFrame(data).to_csv(path / "confidence.csv", index=False)

    def export(self, out_formats, textgrids=True):
        """``textgrids=False``: the TextGrids were already written (infer.py's streaming export)."""
        if textgrids:
            self.save_textgrids()
        if "confidence" in out_formats:
            self.save_confidence_fn()
        if self.log:
            print("error:")
            for line in self.log:
                print(line)
