"""GPU: BASELINE.json's single-GPU configurations at full size, through the
bench's own table and step (bench.Table, one cudasp_scan_device_batches call =
one k_scan_multi launch over every batch).

* config 2: 1M rows, 0 labels, batch_size 300000 (4 batches);
* config 3: 9.4M rows, 1 label (the SQL test's label, test/sql/cudasp.test:104),
  batch_size 300000 (32 batches);
* the config-5 shape on one GPU: 16 labels, 1..15 outputs per row (mean 8),
  11 full 300000-row batches in one launch.

Each asserts found == flagged == planted (every planted base and label value
found, no other row flagged), recomputes the planted values of 256 planted
rows strided over every batch with the C oracle (bench.planted_oracle_check),
and compares the GPU's flags of 512 rows strided over the whole table --
planted or not -- with the oracle's flags for the same rows and outputs.  The
oracle (oracle/) is the checker only."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, ROOT)
    import bench as b
    return b


def strided_flags_check(bench, tab, labels, count=512):
    """GPU flags of `count` rows strided over the table against the oracle's."""
    from oracle import oracle
    tw, outs, offs, lens, gflags = [], [], [], [], []
    base = 0
    step = max(1, tab.rows // count)
    g = 0
    for b in range(tab.nb):
        m = tab.sizes[b]
        idx = [i for i in range((-g) % step, m, step)]
        g += m
        if not idx:
            continue
        x = tab.cols(tab.tx, b)[:, idx].cpu().numpy().view(np.uint32)
        y = tab.cols(tab.ty, b)[:, idx].cpu().numpy().view(np.uint32)
        tw.append(np.ascontiguousarray(np.concatenate([x.T, y.T], axis=1).astype("<u4")).view(np.uint8)
                  .reshape(len(idx), 64))
        of = tab.offs[b][:m].cpu().numpy().view(np.uint32)
        ln = tab.lens[b][:m].cpu().numpy().view(np.uint32)
        ob = tab.outs[b].cpu().numpy()
        for i in idx:
            outs.append(ob[of[i]:of[i] + ln[i]])
            offs.append(base)
            lens.append(ln[i])
            base += int(ln[i])
        gflags.append(tab.flags[b][:m].cpu().numpy()[idx])
    ref, _ = oracle.scan(bench.SCAN_KEY, bench.SPEND_KEY, labels, np.concatenate(tw), np.concatenate(outs),
                         np.array(offs, np.uint32), np.array(lens, np.uint32), threads=8)
    got = np.concatenate(gflags)
    return int(len(got)), int((got == ref).sum()), int(ref.sum())


def run_config(bench, rows, labels_n, outputs_per_row=2, outputs_max=0):
    import torch
    from cudasp_amd import Scanner, _native
    lib = _native.load()
    dev = torch.cuda.current_device()
    labels = bench.label_keys(labels_n)
    batches = bench.rank_batches("rows", rows, 300_000, 0, 1, None)
    gen = torch.cuda.Stream(dev)
    tab = bench.Table(lib, dev, batches, 300_000, outputs_per_row, labels, dev_stream=gen, kmax=outputs_max)
    st = torch.cuda.Stream(dev)
    with Scanner(bench.SCAN_KEY, bench.SPEND_KEY, labels, max_rows=300_000, device=dev) as s:
        descs = bench.multi_descs(tab)
        bench.run_step_multi(tab, s, st, descs)
        torch.cuda.synchronize(dev)
    found = int(tab.match_count.sum().item())
    flagged = int(tab.flags.sum().item())
    return tab, labels, found, flagged


@pytest.mark.parametrize("rows,labels_n", [(1_000_000, 0), (9_400_000, 1)], ids=["config2", "config3"])
def test_single_gpu_configs_full_size(bench, rows, labels_n):
    tab, labels, found, flagged = run_config(bench, rows, labels_n)
    assert tab.nb == -(-rows // 300_000)
    assert found == flagged == tab.expected, (found, flagged, tab.expected)
    if labels_n:
        assert tab.planted_labels == {0}
    chk = bench.planted_oracle_check(tab, labels, threads=8)
    assert chk["rows"] == 256 and chk["equal"] == 256 and chk["batches"] == tab.nb, chk
    n, equal, ref_hits = strided_flags_check(bench, tab, labels)
    assert n >= 500 and equal == n, (n, equal)


def test_sixteen_labels_many_full_batches_one_launch(bench):
    """The config-5 shape over 11 full batches in one persistent launch: every
    label index planted and found, none other flagged, oracle samples equal."""
    tab, labels, found, flagged = run_config(bench, 3_300_000, 16, outputs_max=15)
    assert tab.nb == 11 and all(m == 300_000 for m in tab.sizes)
    assert found == flagged == tab.expected, (found, flagged, tab.expected)
    assert tab.planted_labels == set(range(16))
    chk = bench.planted_oracle_check(tab, labels, threads=8)
    assert chk["equal"] == chk["rows"] == 256 and chk["label_columns"] == list(range(1, 17)), chk
    n, equal, _ = strided_flags_check(bench, tab, labels)
    assert n >= 500 and equal == n, (n, equal)
