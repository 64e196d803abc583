"""AlignmentDecoder.plot (tools/alignment_decoder.py:152-168) and plot_for_valid (tools/plot.py), pinned by the
reference's own figures on the decode golden cases (tests/golden/plot.json / plot.npz, gen_golden.py plot): the
same vertical boundary lines, phone labels (text, position, colour), curves, image and layout.  CPU: the plotting
function on the reference's own inputs, and the per-frame phone index from the reference's decode outputs."""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
matplotlib = pytest.importorskip("matplotlib")
matplotlib.use("Agg")


def figure_data(fig):
    ax1, ax2 = fig.axes
    vl = [float(ln.get_xdata()[0]) for ln in ax1.lines
          if len(ln.get_xdata()) == 2 and ln.get_xdata()[0] == ln.get_xdata()[1]]
    curves1 = [np.asarray(ln.get_ydata(), np.float64) for ln in ax1.lines if len(ln.get_xdata()) != 2]
    return {"vlines": vl,
            "texts": [[t.get_text(), float(t.get_position()[0]), float(t.get_position()[1]), str(t.get_color())]
                      for t in ax1.texts],
            "conf_curve": curves1[0].tolist() if curves1 else [],
            "image_shape": list(ax2.images[0].get_array().shape),
            "bottom_curves": [np.asarray(ln.get_ydata(), np.float64).tolist() for ln in ax2.lines],
            "size": [float(v) for v in fig.get_size_inches()],
            "subplotpars": [fig.subplotpars.left, fig.subplotpars.right, fig.subplotpars.top,
                            fig.subplotpars.bottom, fig.subplotpars.hspace]}


def _golden():
    return json.load(open(os.path.join(GOLD, "plot.json")))["cases"], np.load(os.path.join(GOLD, "plot.npz"))


def test_plot_for_valid_matches_reference_figures():
    import matplotlib.pyplot as plt
    from hubertfa_amd.plot import plot_for_valid
    cases, z = _golden()
    for ci, c in enumerate(cases):
        fig = plot_for_valid(z[f"c{ci}_mel"], c["ph_seq"], z[f"c{ci}_ph_intervals_int"], z[f"c{ci}_frame_confidence"],
                             z[f"c{ci}_ph_frame_prob"], z[f"c{ci}_ph_idx_frame"], z[f"c{ci}_edge_prob"])
        assert figure_data(fig) == c["figure"], ci
        assert np.array_equal(fig.axes[1].images[0].get_array(), z[f"c{ci}_ph_frame_prob"].T)
        plt.close(fig)


def test_phone_index_per_frame_matches_reference():
    """The bottom panel's red line from the decode goldens' path (ph_idx_seq, ph_time_int): the reference's values."""
    from hubertfa_amd.plot import phone_index_per_frame
    cases, z = _golden()
    dz = np.load(os.path.join(GOLD, "decode_cases.npz"))
    for ci in range(len(cases)):
        T = z[f"c{ci}_ph_frame_prob"].shape[0]
        got = phone_index_per_frame(dz[f"c{ci}_ph_idx_seq"], dz[f"c{ci}_ph_time_int"], T)
        assert np.array_equal(got, z[f"c{ci}_ph_idx_frame"]), ci


@pytest.mark.gpu
def test_decoder_plot_matches_reference():
    """AlignmentDecoder.decode on the GPU, then .plot: the reference's figure (its boundaries, labels and phone-index
    line exactly; the probability image and curves within the lattice's 1e-5)."""
    import matplotlib.pyplot as plt
    import torch
    from hubertfa_amd.alignment_decoder import AlignmentDecoder
    cases, z = _golden()
    d = json.load(open(os.path.join(GOLD, "decode_cases.json")))
    dz = np.load(os.path.join(GOLD, "decode_cases.npz"))
    dec = AlignmentDecoder(d["vocab"], {"hop_length": 512, "sample_rate": 44100})
    for ci, (c, dc) in enumerate(zip(cases, d["cases"])):
        lt = torch.from_numpy(dz[f"c{ci}_logits"]).cuda()
        frame, edge = lt[:, :, 2:], lt[:, :, 0]
        ctc = torch.cat([lt[:, :, [1]], lt[:, :, 3:]], dim=-1)
        dec.decode(frame, edge, ctc, dc["wav_length"], dc["ph_seq"], dc["word_seq"], dc["ph_idx_to_word_idx"])
        fig = dec.plot(torch.from_numpy(z[f"c{ci}_mel"]))
        got, ref = figure_data(fig), c["figure"]
        assert got["vlines"] == ref["vlines"] and got["image_shape"] == ref["image_shape"], ci
        assert [t[0] for t in got["texts"]] == [t[0] for t in ref["texts"]], ci
        np.testing.assert_allclose([t[1:3] for t in got["texts"]], [t[1:3] for t in ref["texts"]], atol=1e-9)
        assert got["bottom_curves"][0] == ref["bottom_curves"][0], ci            # the phone index per frame
        np.testing.assert_allclose(got["conf_curve"], ref["conf_curve"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(got["bottom_curves"][1], ref["bottom_curves"][1], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(fig.axes[1].images[0].get_array(), z[f"c{ci}_ph_frame_prob"].T, atol=1e-5)
        plt.close(fig)
