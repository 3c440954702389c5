"""THCM options the device library does not restate are refused by name before any device
work (VERDICT r05 missing #3: THCM::fixPressurePoints, THCM.C:2201-2238, default false at
THCM.C:2792)."""
import pytest

from iemic import config as cf


def test_fix_pressure_points_refused_by_name():
    c = cf.preset("natl8").with_(fix_pressure_points=True)
    with pytest.raises(NotImplementedError, match="Fix Pressure Points"):
        c.validate()


def test_default_config_validates():
    for name in ("natl8", "gateway16", "global2"):
        cf.preset(name).validate()


def test_ocean_refuses_before_touching_the_device():
    from iemic.ocean import Ocean
    c = cf.preset("natl8").with_(fix_pressure_points=True)
    with pytest.raises(NotImplementedError, match="fixPressurePoints"):
        Ocean(c)
