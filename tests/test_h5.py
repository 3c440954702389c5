"""State files in the reference's HDF5 layout (iemic.h5; Model::saveStateToFile /
loadStateFromFile, src/utils/Model.H:149-330)."""
import os

import numpy as np
import pytest

from helpers import golden
from iemic import h5

REF_H5 = "/root/reference/test/ocean/ocean_reference.h5"


def test_roundtrip(tmp_path):
    rng = np.random.default_rng(2)
    tree = {"State": {"Values": rng.standard_normal((1, 1000)),
                      "GlobalLength": np.array(1000, dtype=np.int32),
                      "__type__": np.array([b"Epetra_MultiVector"], dtype="S19")},
            "Parameters": {f"P{i}": np.array(float(i) * 0.5) for i in range(40)},
            "Grid": {"x": np.linspace(0, 1, 7), "n": np.array(7, dtype=np.int32),
                     "mask": (np.arange(30, dtype=np.int32) % 3), "nested": {"k": np.arange(4.0)}},
            "scalar": np.array(3.25)}
    p = str(tmp_path / "t.h5")
    h5.write(p, tree)
    t = h5.read(p)
    np.testing.assert_array_equal(t["/State/Values"][0], tree["State"]["Values"])
    assert t["/State/GlobalLength"][0] == 1000 and t["/State/GlobalLength"][0].dtype == np.int32
    assert t["/State/__type__"][0][0] == b"Epetra_MultiVector"
    for i in range(40):
        assert t[f"/Parameters/P{i}"][0] == i * 0.5
    np.testing.assert_array_equal(t["/Grid/mask"][0], tree["Grid"]["mask"])
    np.testing.assert_array_equal(t["/Grid/nested/k"][0], np.arange(4.0))
    assert t["/scalar"][0] == 3.25
    assert open(p, "rb").read(8) == b"\x89HDF\r\n\x1a\n"


@pytest.mark.skipif(not os.path.exists(REF_H5), reason="reference tree absent (GPU box)")
def test_reads_reference_state_file():
    """the reference's own test/ocean/ocean_reference.h5 (written by EpetraExt::HDF5):
    its state equals the byte-offset decode committed in tests/golden/gateway16.npz"""
    t = h5.read(REF_H5)
    np.testing.assert_array_equal(t["/State/Values"][0][0], golden("gateway16")["h5_x"])
    assert t["/State/GlobalLength"][0] == 24576
    assert abs(t["/Parameters/Combined Forcing"][0] - 0.02) < 1e-6
    assert t["/MaskGlobal/Global"][0].size == 18 ** 3


@pytest.mark.gpu
def test_ocean_save_load_roundtrip(tmp_path):
    from iemic import config as cf
    from iemic.ocean import Ocean
    from helpers import golden_landm
    c = cf.preset("gateway16")
    oc = Ocean(c, landm=golden_landm("gateway16"))
    x = golden("gateway16")["h5_x"]
    oc.setState(x)
    oc.setPar("Combined Forcing", 0.02)
    p = str(tmp_path / "ocean.h5")
    oc.saveStateToFile(p)
    oc2 = Ocean(c, landm=golden_landm("gateway16"))
    assert oc2.loadStateFromFile(p) == 0
    np.testing.assert_array_equal(oc2.getState(), x)
    assert oc2.getPar("Combined Forcing") == 0.02
    np.testing.assert_array_equal(oc2.computeRHS(), oc.computeRHS())
    assert oc2.loadStateFromFile(str(tmp_path / "missing.h5")) == 1
