"""GPU CSV reader (csrc/csv.hip, prep/csv_gpu.py) vs the pyarrow reader it replaces (run with -m gpu)."""
import numpy as np
import pytest
import torch

from cobalt_smart_lender_ai_amd.prep.device_frame import DeviceFrame

pytestmark = pytest.mark.gpu


def _decoded(frame, name):
    c = frame[name]
    if c.kind == "c":
        codes = c.data.cpu().numpy()
        return [c.vocab[k] if k >= 0 else None for k in codes]
    return frame.host_strings(name).to_pylist()


def assert_frames_identical(a: DeviceFrame, b: DeviceFrame):
    assert a.columns == b.columns
    assert a.n == b.n
    for name in a.columns:
        ca, cb = a[name], b[name]
        assert (ca.kind in "ch") == (cb.kind in "ch"), name
        assert ca.dtype == cb.dtype, (name, ca.dtype, cb.dtype)
        if ca.kind in "ch":
            assert ca.kind == cb.kind, name
            assert _decoded(a, name) == _decoded(b, name), name
        elif ca.kind == "f":
            x, y = ca.data.cpu().numpy(), cb.data.cpu().numpy()
            nx, ny = np.isnan(x), np.isnan(y)
            assert np.array_equal(nx, ny), name
            assert np.array_equal(x[~nx].view(np.int64), y[~ny].view(np.int64)), name  # bitwise, incl. -0.0
        else:
            assert ca.kind == cb.kind and torch.equal(ca.data, cb.data), name


def _tricky_csv(n: int, seed: int, crlf: bool) -> bytes:
    rng = np.random.default_rng(seed)
    nl = "\r\n" if crlf else "\n"
    words = ["alpha", "beta", "Gamma, Inc.", 'say "hi"', "multi\nline", "ünïcødé", "NA", "", "x"]
    rows = ['id,name,amount,flag,flag_null,note,empty,mixed,intnull,big,expo,neg0,plus,uniq,"quoted, header"']
    for i in range(n):
        def q(s):
            return '"' + s.replace('"', '""') + '"' if any(ch in s for ch in ',"\n') or rng.random() < 0.1 else s
        amount = rng.choice([f"{rng.normal() * 1e4:.4f}", "", "NaN", "-0.0", f"{rng.integers(-99, 99)}", "1.5e-3"])
        rows.append(",".join([
            str(i),
            q(str(rng.choice(words))),
            amount,
            str(rng.choice(["True", "False", "true", "FALSE"])),
            str(rng.choice(["True", "False", ""])),
            q(f"note {rng.integers(0, 50)}, {rng.choice(words)}"),
            "",
            str(rng.choice(["12", "abc", "3.5", ""])),
            str(rng.choice(["7", "", "-0", "123"])),
            str(rng.choice(["123456789012345678901234", "5", "9007199254740993"])),
            str(rng.choice(["1e3", "2.5E+2", "-7e-2", "0.1"])),
            "-0",
            str(rng.choice(["+5", "6"])),
            q(f"user-{rng.integers(0, 1 << 40):x}, {i}"),
            str(rng.choice(["12.5", "7"])),
        ]))
    return (nl.join(rows) + nl).encode("utf-8")


@pytest.mark.parametrize("crlf", [False, True])
def test_tricky_csv_matches_pyarrow(crlf):
    data = _tricky_csv(3001, 3 + crlf, crlf)
    t = {}
    g = DeviceFrame.read_csv(data, "cuda", engine="gpu", timings=t)
    a = DeviceFrame.read_csv(data, "cuda", engine="arrow")
    assert t["rows"] == 3001 and t["cols"] == 15
    assert_frames_identical(g, a)
    assert g["uniq"].kind == "h" and g["name"].kind == "c"
    assert g["neg0"].dtype == "int64" and g["plus"].dtype == "float64" and g["big"].dtype == "float64"
    assert g["flag"].kind == "b" and g["flag_null"].dtype == "boolnull"


def test_no_trailing_newline_and_small_frame():
    data = b'a,b,c\n1,"x,y",2.5\n2,,3'
    g = DeviceFrame.read_csv(data, "cuda", engine="gpu")
    a = DeviceFrame.read_csv(data, "cuda", engine="arrow")
    assert_frames_identical(g, a)
    assert g.n == 2 and g["b"].kind == "c"


def test_ragged_file_falls_back():
    from cobalt_smart_lender_ai_amd.prep.csv_gpu import CsvLayoutError

    data = b"a,b\n1,2\n3\n4,5\n"
    with pytest.raises(CsvLayoutError):
        DeviceFrame.read_csv(data, "cuda", engine="gpu")
    auto = DeviceFrame.read_csv(b"a,b\n1,2\n\n3,4\n", "cuda")  # blank line: pyarrow fallback
    assert auto.n == 2


def test_synthetic_raw_lendingclub_matches_pyarrow(tmp_path):
    from cobalt_smart_lender_ai_amd.dataio.synth_raw import make_raw_lendingclub

    df = make_raw_lendingclub(200_000, seed=5, n_cols=143)
    path = tmp_path / "raw.csv"
    df.to_csv(path, index=False)
    t = {}
    g = DeviceFrame.read_csv(str(path), "cuda", engine="gpu", timings=t)
    a = DeviceFrame.read_csv(str(path), "cuda", engine="arrow")
    assert t["cols"] == 143
    assert_frames_identical(g, a)


# ------------------------------------------------------------------------------------------ writer
def _pandas_bytes(frame) -> bytes:
    return frame.to_pandas().to_csv(index=False).encode("utf-8")


def test_writer_floats_all_magnitudes_match_pandas():
    from cobalt_smart_lender_ai_amd.prep.csv_gpu import frame_to_csv_bytes
    from cobalt_smart_lender_ai_amd.prep.device_frame import DCol

    rng = np.random.default_rng(11)
    n = 200_000
    mags = rng.normal(size=n) * 10.0 ** rng.uniform(-30, 30, n)
    sc = 10.0 ** rng.integers(0, 6, n)
    short = np.round(rng.normal(size=n) * 1000 * sc) / sc  # "nice" decimals
    ints = rng.integers(-10**15, 10**15, n).astype(np.float64)
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e16, 1e15, 0.0001, 1e-05, 9999999999999998.0,
                        1.7976931348623157e308, 2.2250738585072014e-288, 0.1, 1 / 3, 123456789.123, 5e-5] * (n // 16))
    mk = lambda a, dt="float64": DCol("f", torch.as_tensor(a, device="cuda"), dt)  # noqa: E731
    fr = DeviceFrame({"mags": mk(mags), "short": mk(short), "ints": mk(ints, "int64"), "special": mk(special),
                      "intnan": mk(np.where(rng.random(n) < 0.1, np.nan, ints), "int64")}, n, "cuda")
    t = {}
    got = frame_to_csv_bytes(fr, timings=t)
    assert got is not None
    got = bytes(got)
    want = _pandas_bytes(fr)
    if got != want:  # locate the first differing line for the failure message
        g, w = got.split(b"\n"), want.split(b"\n")
        i = next(i for i in range(min(len(g), len(w))) if g[i] != w[i])
        raise AssertionError(f"line {i}: gpu {g[i]!r} pandas {w[i]!r}")


def test_writer_strings_codes_flags_and_row_filter_match_pandas():
    from cobalt_smart_lender_ai_amd.prep.csv_gpu import frame_to_csv_bytes

    data = _tricky_csv(4001, 9, crlf=True)
    fr = DeviceFrame.read_csv(data, "cuda", engine="gpu")
    assert bytes(frame_to_csv_bytes(fr)) == _pandas_bytes(fr)
    keep = torch.as_tensor(np.random.default_rng(2).random(fr.n) < 0.6, device="cuda")
    sub = fr.take(keep)
    assert bytes(frame_to_csv_bytes(sub)) == _pandas_bytes(sub)
    arrow_fr = DeviceFrame.read_csv(data, "cuda", engine="arrow")  # text kept as Arrow columns
    assert bytes(frame_to_csv_bytes(arrow_fr.take(keep))) == _pandas_bytes(arrow_fr.take(keep))


def test_writer_prep_outputs_match_pandas(tmp_path):
    from cobalt_smart_lender_ai_amd.dataio.synth_raw import make_raw_lendingclub
    from cobalt_smart_lender_ai_amd.prep import device_prep as dp
    from cobalt_smart_lender_ai_amd.prep.csv_gpu import frame_to_csv_bytes

    path = tmp_path / "raw.csv"
    make_raw_lendingclub(60_000, seed=3, n_cols=143).to_csv(path, index=False)
    res = dp.run_device_prep(str(path), device="cuda", reference_date="2025-07-04")
    for key in ("clean", "tree", "nn"):
        assert bytes(frame_to_csv_bytes(res[key])) == _pandas_bytes(res[key]), key


def test_writer_splices_host_formatted_values():
    from cobalt_smart_lender_ai_amd.prep.csv_gpu import frame_to_csv_bytes
    from cobalt_smart_lender_ai_amd.prep.device_frame import DCol

    x = [1.0, 5e-324, -2.5e-310, 1.7976931348623157e308, -1e300, 0.1, float("nan"), 4.9e-321]
    fr = DeviceFrame({"x": DCol("f", torch.tensor(x, dtype=torch.float64, device="cuda"), "float64"),
                      "y": DCol("f", torch.arange(8, dtype=torch.float64, device="cuda"), "int64")}, 8, "cuda")
    assert bytes(frame_to_csv_bytes(fr)) == _pandas_bytes(fr)


def test_read_table_equals_pandas_read_csv(tmp_path):
    """The train / train-nn CLI input read on the GPU equals pandas' correctly rounded reader."""
    import io

    import pandas as pd

    from cobalt_smart_lender_ai_amd.dataio.artifacts import LocalStore
    from cobalt_smart_lender_ai_amd.dataio.synth_raw import make_raw_lendingclub
    from cobalt_smart_lender_ai_amd.pipeline.prep_flow import read_table
    from cobalt_smart_lender_ai_amd.prep import device_prep as dp
    from cobalt_smart_lender_ai_amd.prep.csv_gpu import frame_to_csv_bytes

    path = tmp_path / "raw.csv"
    make_raw_lendingclub(30_000, seed=8, n_cols=143).to_csv(path, index=False)
    res = dp.run_device_prep(str(path), device="cuda", reference_date="2025-07-04")
    st = LocalStore(tmp_path / "lake")
    for key in ("tree", "nn"):
        st.put_bytes(f"{key}.csv", frame_to_csv_bytes(res[key]))
        got = read_table(st, f"{key}.csv", "cuda")
        # what the reference's job reads: pandas' DEFAULT float conversion, reproduced on the device
        want = pd.read_csv(io.BytesIO(st.get_bytes(f"{key}.csv")), low_memory=False)
        pd.testing.assert_frame_equal(got, want, check_exact=True)
        assert got.equals(st.read_csv(f"{key}.csv"))  # = the CPU path of read_table


def test_prep_flow_gpu_engine_writes_the_pandas_artifacts(tmp_path):
    """Both CLI prep stages on the GPU (GPU CSV reader -> device stages -> GPU CSV writer) save the
    same artifacts as the pandas engine (values equal up to pandas' own parser rounding)."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).parent))
    from test_device_prep import REF_DATE, assert_frames_equal

    from cobalt_smart_lender_ai_amd.config import CLEAN_DATA_KEY_FULL, CLEAN_DATA_KEY_NN, CLEAN_DATA_KEY_TREE, \
        RAW_DATA_KEY_FULL
    from cobalt_smart_lender_ai_amd.dataio.artifacts import LocalStore
    from cobalt_smart_lender_ai_amd.dataio.synth_raw import make_raw_lendingclub
    from cobalt_smart_lender_ai_amd.pipeline.prep_flow import run_clean, run_features

    raw = make_raw_lendingclub(20_000, seed=21, n_cols=143)
    outs = {}
    for tag, engine, dev in (("pandas", "pandas", "cpu"), ("device_cpu", "device", "cpu"), ("gpu", "device", "cuda")):
        st = LocalStore(tmp_path / tag)
        st.write_csv(raw, RAW_DATA_KEY_FULL)
        run_clean(st, use_sample=False, device=dev, engine=engine)
        run_features(st, device=dev, reference_date=REF_DATE, engine=engine)
        outs[tag] = [st.read_csv(k, float_precision="round_trip")
                     for k in (CLEAN_DATA_KEY_FULL, CLEAN_DATA_KEY_TREE, CLEAN_DATA_KEY_NN)]
    # the GPU engine (GPU reader + kernels + GPU writer) vs the same stages on CPU tensors (pyarrow
    # reader, pandas writer): equal up to the last ulp of device vs host log1p
    for a, b in zip(outs["gpu"], outs["device_cpu"]):
        assert_frames_equal(a, b, rtol=1e-15)
    # vs the pandas engine: pandas' default float parser reads some raw values a few dozen ulp off
    for a, b in zip(outs["gpu"], outs["pandas"]):
        assert_frames_equal(a, b, rtol=1e-13)


def test_gpu_reader_pandas_typing_duplicates_and_nullable_bools():
    """read_table's GPU path equals pandas.read_csv on repeated headers (a, a.2, ...) and nullable
    bools (object True / False / NaN), and the GPU writer renders that frame as pandas.to_csv does."""
    import io

    import pandas as pd

    from cobalt_smart_lender_ai_amd.prep.csv_gpu import frame_to_csv_bytes

    data = b"a,b,a,flag,flagn,a.1\n1,x,2.5,True,True,7\n2,y,3.5,False,,8\n3,,4.5,True,False,9\n"
    ref = pd.read_csv(io.BytesIO(data), float_precision="round_trip")
    g = DeviceFrame.read_csv(data, "cuda", engine="gpu")
    pd.testing.assert_frame_equal(g.to_pandas(), ref)
    assert bytes(frame_to_csv_bytes(g)) == ref.to_csv(index=False).encode()


def _float_strings(n=20000, seed=1):
    import random

    rng = random.Random(seed)
    out = []
    for _ in range(n):
        k = rng.randint(0, 7)
        if k == 0:
            s = repr(float(np.float32(rng.uniform(0, 1000))))  # 17-digit float32 values (the API's echo)
        elif k == 1:
            s = repr(rng.uniform(-1e6, 1e6))
        elif k == 2:
            s = "0.0000" + "".join(rng.choice("0123456789") for _ in range(rng.randint(1, 22)))
        elif k == 3:
            s = ("".join(rng.choice("0123456789") for _ in range(rng.randint(1, 25))) + "." +
                 "".join(rng.choice("0123456789") for _ in range(rng.randint(1, 10))))
        elif k == 4:
            s = repr(rng.uniform(0, 1) * 10 ** rng.randint(-30, 30))
        elif k == 5:
            s = "%.20e" % rng.uniform(1, 10)
        elif k == 6:
            s = "-" + repr(rng.uniform(0, 1) * 10 ** rng.randint(-320, -300))  # subnormal range
        else:
            s = "00" + repr(rng.uniform(0, 100))
        out.append(s)
    return out


def test_pandas_default_float_conversion_bit_exact():
    """float_precision="high" reproduces pandas.read_csv's DEFAULT float conversion (not correctly
    rounded: 17 leading digits accumulated in double, one scale by 10^k) bit for bit; "round_trip"
    equals pandas' round_trip mode. The strings include 17-digit float32 reprs, leading zeros, > 17
    digits, exponents and subnormals."""
    import io

    import pandas as pd

    strs = _float_strings()
    body = ("x,y\n" + "\n".join(f"{s},{i}" for i, s in enumerate(strs)) + "\n").encode()
    want_hi = pd.read_csv(io.BytesIO(body))["x"].to_numpy()
    want_rt = pd.read_csv(io.BytesIO(body), float_precision="round_trip")["x"].to_numpy()
    assert (want_hi != want_rt).sum() > 100  # the two pandas modes do differ on these strings
    hi = DeviceFrame.read_csv(body, "cuda", engine="gpu", float_precision="high")
    rt = DeviceFrame.read_csv(body, "cuda", engine="gpu")
    got_hi, got_rt = hi["x"].data.cpu().numpy(), rt["x"].data.cpu().numpy()
    assert np.array_equal(got_hi.view(np.int64), want_hi.view(np.int64))
    assert np.array_equal(got_rt.view(np.int64), want_rt.view(np.int64))
    # an overflow is text to pandas: the device reader refuses the file instead of guessing
    with pytest.raises(Exception):
        DeviceFrame.read_csv(b"x\n1e400\n1.5\n", "cuda", engine="gpu", float_precision="high")
