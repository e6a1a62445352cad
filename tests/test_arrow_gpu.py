"""GPU: the columnar (Arrow) input path, cudasp_tf_function_columns behind
cudasp_scan_arrow.  It must give exactly the row
path's results (cudasp_scan, itself checked against the reference's SQL file
and the oracle): same SQL-file queries, NULL rules, sliced arrays with
offsets, fixed-size and variable binary tweaks, large types, batch
boundaries, and the tweak-length error."""
import pytest

import golden_io

pytestmark = pytest.mark.gpu
pa = pytest.importorskip("pyarrow")


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _arrow(rows, tweak_type=None, large=False):
    txid, height, tweak, outs = zip(*rows) if rows else ([], [], [], [])
    bin_t = pa.large_binary() if large else pa.binary()
    list_t = pa.large_list(pa.int64()) if large else pa.list_(pa.int64())
    return pa.table({
        "txid": pa.array(list(txid), bin_t),
        "height": pa.array(list(height), pa.int32()),
        "tweak_key": pa.array(list(tweak), tweak_type or bin_t),
        "outputs": pa.array(list(outs), list_t),
    })


def _rows(tbl):
    d = tbl.to_pydict()
    return sorted(zip(d["txid"], d["height"], d["tweak_key"]))


def _sql_table(sc, q):
    if q["table"] == "test_data":
        rows = sc["tables"]["test_data"][:q["test_data_rows_visible"]]
        rows = [r for r in rows if q["where_height"] in (None, r["height"])]
        return [(bytes.fromhex(r["txid"]), r["height"], bytes.fromhex(r["tweak"]), r["outputs"]) for r in rows]
    t = sc["tables"][q["table"]]
    r = t["row"]
    return [(bytes.fromhex(r["txid"]), r["height"], bytes.fromhex(r["tweak"]), r["outputs"])] * t["repeat"]


@pytest.mark.parametrize("threads", [1, 3])
def test_sql_file_columnar(gpu, threads):
    from cudasp_amd import cudasp_scan, cudasp_scan_arrow
    sc = golden_io.load("sql_cases.json")
    for q in sc["queries"]:
        rows = _sql_table(sc, q)
        keys = (bytes.fromhex(q["scan_key"]), bytes.fromhex(q["spend_key"]), [bytes.fromhex(l) for l in q["label_keys"]])
        out = cudasp_scan_arrow(_arrow(rows), *keys, batch_size=q["batch_size"], threads=threads, piece_rows=1000)
        want = cudasp_scan(rows, *keys, batch_size=q["batch_size"], threads=threads)
        assert _rows(out) == sorted(want), q["line"]
        got = [out.num_rows] if q["select"] == "count" else sorted(out.column("height").to_pylist())
        assert got == q["expected"], (q["line"], got)


def test_nulls_slices_and_types(gpu):
    from cudasp_amd import cudasp_scan, cudasp_scan_arrow
    sc = golden_io.load("sql_cases.json")
    q = sc["queries"][2]
    r = [x for x in sc["tables"]["test_data"] if x["height"] == 200][0]
    tw, txid, v = bytes.fromhex(r["tweak"]), bytes.fromhex(r["txid"]), r["outputs"][0]
    keys = (bytes.fromhex(q["scan_key"]), bytes.fromhex(q["spend_key"]), [])
    rows = [
        (txid, 1, tw, [v]), (None, 2, tw, [v]), (txid, None, tw, [v]), (txid, 4, None, [v]),
        (txid, 5, tw, None), (txid, 6, tw, [None, v]), (txid, 7, tw, []), (b"", 8, tw, [v, v]),
    ] * 50
    want = sorted(cudasp_scan(rows, *keys))
    assert sorted(h for _, h, _ in want)[:3] == [1, 1, 1]
    for tweak_type in (None, pa.binary(64)):
        for large in (False, True):
            if large and tweak_type is not None:
                continue
            tbl = _arrow(rows, tweak_type, large)
            assert _rows(cudasp_scan_arrow(tbl, *keys)) == want
            # a slice (non-zero array offsets in every column, child included)
            sl = tbl.slice(37, 250)
            assert _rows(cudasp_scan_arrow(sl, *keys)) == sorted(cudasp_scan(rows[37:287], *keys))
    assert cudasp_scan_arrow(_arrow([]), *keys).num_rows == 0


def test_batch_boundaries_and_pieces(gpu):
    from cudasp_amd import cudasp_scan, cudasp_scan_arrow
    rr = golden_io.load("random_rows.json")
    rows = [(i.to_bytes(32, "big"), i, bytes.fromhex(x["tweak"]), x["outputs"]) for i, x in enumerate(rr["rows"])]
    rows = rows * 40  # 5120 rows
    keys = (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), [bytes.fromhex(l) for l in rr["label_keys"]])
    want = sorted(cudasp_scan(rows, *keys))
    assert want
    tbl = _arrow(rows)
    for bs, piece in ((1, 4096), (7, 333), (2048, 2048), (2049, 10000), (300000, 1000)):
        assert _rows(cudasp_scan_arrow(tbl, *keys, batch_size=bs, piece_rows=piece, threads=2)) == want, bs


def test_record_batch_stream(gpu):
    """An iterable of record batches (e.g. a Parquet reader) works the same."""
    from cudasp_amd import cudasp_scan, cudasp_scan_arrow
    rr = golden_io.load("random_rows.json")
    rows = [(i.to_bytes(32, "big"), i, bytes.fromhex(x["tweak"]), x["outputs"]) for i, x in enumerate(rr["rows"])]
    keys = (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), [bytes.fromhex(l) for l in rr["label_keys"]])
    batches = _arrow(rows).to_batches(max_chunksize=17)
    assert _rows(cudasp_scan_arrow(iter(batches), *keys)) == sorted(cudasp_scan(rows, *keys))


def test_parquet_file(gpu, tmp_path):
    """The reference's README shape, cudasp_scan(read_parquet(...), ...)
    (README.md:109 there): a Parquet file written and read back by pyarrow
    (several row groups, fixed_size_binary tweaks, NULLs), streamed as the
    reader's record batches and read whole, equals the row path."""
    pq = pytest.importorskip("pyarrow.parquet")
    from cudasp_amd import cudasp_scan, cudasp_scan_arrow
    rr = golden_io.load("random_rows.json")
    rows = [(i.to_bytes(32, "big"), 900000 + i, bytes.fromhex(x["tweak"]), x["outputs"]) for i, x in enumerate(rr["rows"])]
    rows = rows * 8
    rows[5] = (rows[5][0], rows[5][1], rows[5][2], None)
    rows[9] = (None,) + rows[9][1:]
    keys = (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), [bytes.fromhex(l) for l in rr["label_keys"]])
    want = sorted(cudasp_scan(rows, *keys))
    assert want
    path = str(tmp_path / "tweaks.parquet")
    pq.write_table(_arrow(rows, pa.binary(64)), path, row_group_size=300)
    f = pq.ParquetFile(path)
    assert f.metadata.num_row_groups > 1
    assert _rows(cudasp_scan_arrow(f.iter_batches(batch_size=250), *keys, batch_size=700, threads=2)) == want
    assert _rows(cudasp_scan_arrow(pq.read_table(path), *keys)) == want


def test_bad_tweak_length(gpu):
    from cudasp_amd import CudaspError, cudasp_scan_arrow
    rr = golden_io.load("random_rows.json")
    rows = [(b"t", 1, bytes.fromhex(rr["rows"][0]["tweak"]), [1]), (b"u", 2, b"\x01" * 63, [1])]
    with pytest.raises(CudaspError, match="64 bytes"):
        cudasp_scan_arrow(_arrow(rows), bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), [])
