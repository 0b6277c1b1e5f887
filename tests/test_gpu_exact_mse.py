"""GPU parity of the exact-order MSE option (mdg_settings.options &
MDG_OPTION_EXACT_MSE, include/mdgpu.h): with it the MSE is compute_mse
(deconvoluter.rs:828-862) in the reference's operation order, so it must equal the
oracle's (goldens: oracle outputs) BIT FOR BIT -- not within MSE_RTOL -- on every
golden case, in batches, through the Python surface and the spectrum queue; the
Lorentzians, counts and statuses are the same as without it."""
import os

import numpy as np
import pytest

import oracle
from tests.conftest import GOLDEN
from tests.golden.cases import CASES, load_case, synth_spectrum
from tests.test_gpu_parity import gpu_batch

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("metabodecon._native")


@pytest.fixture(scope="module")
def ctx():
    return nat.context(0)


def exact(settings):
    s = nat.Settings()
    for f, _ in nat.Settings._fields_:
        setattr(s, f, getattr(settings, f))
    s.options = nat.OPTION_EXACT_MSE
    return s


@pytest.mark.parametrize("name", CASES)
def test_exact_mse_golden_cases(ctx, name):
    g = np.load(os.path.join(GOLDEN, "expected", f"{name}.npz"))
    x, y, sb, st, ign = load_case(name)
    status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], exact(st), ign)
    assert status[0] == int(g["status"]), name
    if status[0]:
        return
    assert counts[0] == g["params"].shape[0]
    assert np.array_equal(out[0, : counts[0]], g["params"])
    assert mse[0] == float(g["mse"]), (name, mse[0], float(g["mse"]))


def test_exact_mse_batches(ctx):
    """The 16 blood spectra in one batch and three synthetic spectra with different
    peak counts (the residual rows and region folds per spectrum)."""
    names = [f"blood_{i:02d}" for i in range(1, 17)]
    data = [load_case(n) for n in names]
    status, counts, out, mse = gpu_batch(ctx, np.stack([d[0] for d in data]),
                                         np.stack([d[1] for d in data]), [d[2] for d in data],
                                         exact(data[0][3]))
    for k, n in enumerate(names):
        g = np.load(os.path.join(GOLDEN, "expected", f"{n}.npz"))
        assert status[k] == 0 and np.array_equal(out[k, : counts[k]], g["params"]), n
        assert mse[k] == float(g["mse"]), n
    rows, ref = [], []
    for seed in (6, 7, 8):
        x, y = synth_spectrum(seed, n=65536, n_peaks=500 + 400 * (seed - 6))[:2]
        rows.append(y)
        ref.append(oracle.deconvolute(x, y, (11.8, -2.2), threads=8))
    status, counts, out, mse = gpu_batch(ctx, x, np.stack(rows), [(11.8, -2.2)],
                                         exact(oracle.default_settings()))
    for s, o in enumerate(ref):
        assert status[s] == o.status == 0
        assert np.array_equal(out[s, : counts[s]], o.params) and mse[s] == o.mse, s


def test_exact_mse_python_surface_and_serde(tmp_path):
    """Deconvoluter.exact_mse: Deconvolution.mse and the mse of write_json /
    write_bin (serialized_deconvolution.rs:18-31) are the reference's bits; the
    option is off by default and the default MSE stays within 1e-12."""
    import metabodecon as md
    spectra = md.Spectrum.read_bruker_set(os.path.join(GOLDEN, "bruker", "blood"), 10, 10,
                                          (-2.2, 11.8))
    dec = md.Deconvoluter()
    assert dec.exact_mse is False
    dec.exact_mse = True
    assert dec.exact_mse is True and dec.settings.options == nat.OPTION_EXACT_MSE
    decs = dec.par_deconvolute_spectra(spectra)
    one = dec.deconvolute_spectrum(spectra[3])
    for k, d in enumerate(decs):
        g = np.load(os.path.join(GOLDEN, "expected", f"blood_{k + 1:02d}.npz"))
        assert np.array_equal(d.params, g["params"]) and d.mse == float(g["mse"]), k
    assert one.mse == decs[3].mse
    decs[0].write_json(str(tmp_path / "d.json"))
    decs[0].write_bin(str(tmp_path / "d.bin"))
    for back in (md.Deconvolution.read_json(str(tmp_path / "d.json")),
                 md.Deconvolution.read_bin(str(tmp_path / "d.bin"))):
        assert back.mse == decs[0].mse
    dec.exact_mse = False
    d0 = dec.deconvolute_spectrum(spectra[0])
    assert abs(d0.mse - decs[0].mse) <= 1e-12 * abs(decs[0].mse)


def test_exact_mse_in_queue_and_ignore_regions():
    """The option travels with the queue's settings; two ignore regions (three MSE
    regions, folded separately, summed in order) on an increasing axis."""
    torch = pytest.importorskip("torch")
    x, y, sb, st, ign = load_case("blood_02_two_regions_increasing")
    g = np.load(os.path.join(GOLDEN, "expected", "blood_02_two_regions_increasing.npz"))
    n = y.size
    xd = torch.from_numpy(x).cuda()
    yd = torch.from_numpy(np.stack([y, y, y])).cuda()
    cap = n // 2 + 2
    out = torch.zeros((3, cap, 3), dtype=torch.float64, device="cuda")
    cnt = torch.zeros(3, dtype=torch.int32, device="cuda")
    mse = torch.zeros(3, dtype=torch.float64, device="cuda")
    status = torch.full((3,), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ig = np.asarray(ign, dtype=np.float64).reshape(-1)
    q = nat.SpectrumQueue(0, n, 2, 2, exact(st), ig)
    try:
        for k in range(3):
            q.submit(xd.data_ptr(), yd[k].data_ptr(), sb, out[k].data_ptr(), cap,
                     cnt[k:].data_ptr(), mse[k:].data_ptr(), status[k:].data_ptr())
        q.synchronize()
    finally:
        q.close()
    for k in range(3):
        assert int(status[k]) == 0 and np.array_equal(out[k, : int(cnt[k])].cpu().numpy(), g["params"])
        assert float(mse[k]) == float(g["mse"])
