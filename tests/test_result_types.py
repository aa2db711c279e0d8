"""A18 result types on the host (no GPU): energies in the reference's summation order.

MultiLevelMODWTResultImpl.computeEnergy (:211-216) sums ``energy += c * c`` left to right and
getTotalEnergy (:109-117) adds the approximation energy first, then levels 1..J; the mutable impl
(MutableMultiLevelMODWTResultImpl.java:176-187) does the same.  A pairwise or dot-product sum differs in
the last bits on most inputs, so the test data is chosen where it does."""
import numpy as np

from vectorwave_amd.modwt import MultiLevelMODWTResult, MutableMultiLevelMODWTResult


def _java_energy(c):
    e = 0.0
    for v in c:
        e += v * v   # Python floats: IEEE binary64, one rounding per operation, as Java
    return e


def _data(J=4, n=3001, seed=5):
    rng = np.random.default_rng(seed)
    # wide dynamic range: sequential and pairwise sums disagree in the last bits
    det = rng.standard_normal((J, n)) * np.exp(rng.uniform(-8, 8, (J, n)))
    app = rng.standard_normal(n) * np.exp(rng.uniform(-8, 8, n))
    return det, app


def test_energies_sequential_like_the_reference():
    det, app = _data()
    for cls in (MultiLevelMODWTResult, MutableMultiLevelMODWTResult):
        r = cls(det.copy(), app.copy())
        assert r.getApproximationEnergy() == _java_energy(app.tolist())
        for j in range(1, det.shape[0] + 1):
            assert r.getDetailEnergyAtLevel(j) == _java_energy(det[j - 1].tolist())
        total = _java_energy(app.tolist())
        for j in range(det.shape[0]):
            total += _java_energy(det[j].tolist())
        assert r.getTotalEnergy() == total


def test_sequential_order_matters_on_this_data():
    # guard that the data above can tell the orders apart (else the test above proves nothing)
    det, app = _data()
    rows = [app] + list(det)
    assert any(float(np.dot(a, a)) != _java_energy(a.tolist()) for a in rows)


def test_relative_distribution_orders():
    det, app = _data(J=3, n=257, seed=9)
    imm = MultiLevelMODWTResult(det.copy(), app.copy())
    mut = MutableMultiLevelMODWTResult(det.copy(), app.copy())
    tot = imm.getTotalEnergy()
    ea = _java_energy(app.tolist())
    ed = [_java_energy(det[j].tolist()) for j in range(3)]
    # immutable: [approx, d1..dJ] (MultiLevelMODWTResultImpl.java:121-138); mutable: [d1..dJ, approx]
    assert imm.getRelativeEnergyDistribution() == [ea / tot] + [e / tot for e in ed]
    assert mut.getRelativeEnergyDistribution() == [e / tot for e in ed] + [ea / tot]
    z = MultiLevelMODWTResult(np.zeros((2, 8)), np.zeros(8))
    assert z.getTotalEnergy() == 0.0 and z.getRelativeEnergyDistribution() == [0.0, 0.0, 0.0]
