"""Wavelet filter banks: Python mirror of VectorWave's ``core/api`` wavelet types.

Taps are the reference's literal decimal constants (parsed to the same IEEE doubles as the Java
literals):
  Haar      core/api/Haar.java:39-43           (1/sqrt(2), computed exactly as Java does)
  Daubechies core/api/Daubechies.java:61-165   (DB2..DB10)
  Symlet    core/api/Symlet.java:53-215        (SYM2..SYM8, SYM10)
  Coiflet   core/api/Coiflet.java:38-190       (COIF1..COIF5)
High-pass filters use the QMF relation g[i] = (-1)^i h[L-1-i]
(core/api/Daubechies.java:323-330, Symlet.java:462-469, Coiflet.java:629-636); orthogonal
wavelets reconstruct with their decomposition filters (core/api/OrthogonalWavelet.java:23-35).

``wavelet_id`` carries the object identity the reference's SymmetricAlignmentStrategy tests
(core/modwt/SymmetricAlignmentStrategy.java:65-96) across the C ABI.
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

# wavelet identity codes (include/vectorwave_amd.h)
WID_OTHER, WID_HAAR, WID_DB2, WID_DB4, WID_DB6, WID_DB8, WID_DB10 = 0, 1, 2, 4, 6, 8, 10
WID_SYM4, WID_SYM8 = 104, 108
WID_COIF1, WID_COIF2, WID_COIF3, WID_COIF5 = 201, 202, 203, 205

_SQRT2_INV = 1.0 / math.sqrt(2)  # Haar.java:39

_DB2 = (
        0.4829629131445341, 0.8365163037378079, 0.2241438680420134, -0.1294095225512603,
)
_DB4 = (
        0.2303778133088964, 0.7148465705529154, 0.6308807679298587, -0.0279837693982488,
        -0.1870348117190931, 0.0308413818355607, 0.0328830116668852, -0.0105974017850690,
)
_DB6 = (
        0.1115407433501094, 0.4946238903984530, 0.7511339080210954, 0.3152503517091980,
        -0.2262646939654399, -0.1297668675672624, 0.0975016055873224, 0.0275228655303053,
        -0.0315820393174862, 0.0005538422011614, 0.0047772575109455, -0.0010773010853085,
)
_DB8 = (
        0.0544158422431049, 0.3128715909143031, 0.6756307362972904, 0.5853546836541907,
        -0.0158291052563816, -0.2840155429615702, 0.0004724845739124, 0.1287474266204837,
        -0.0173693010018083, -0.0440882539307952, 0.0139810279173995, 0.0087460940474061,
        -0.0048703529934518, -0.0003917403733770, 0.0006754494064506, -0.0001174767841248,
)
_DB10 = (
        0.0266700579005546, 0.1881768000776347, 0.5272011889317202, 0.6884590394536250,
        0.2811723436605715, -0.2498464243271598, -0.1959462743772862, 0.1273693403357932,
        0.0930573646035547, -0.0713941471663501, -0.0294575368218399, 0.0332126740593612,
        0.0036065535669870, -0.0107331754833007, 0.0013953517470688, 0.0019924052951925,
        -0.0006858566949564, -0.0001164668551285, 0.0000935886703202, -0.0000132642028945,
)
_SYM2 = (
        0.48296291314453414, 0.83651630373780772, 0.22414386804201339, -0.12940952255126034,
)
_SYM3 = (
        0.33267055295095688, 0.80689150931333875, 0.45987750211933132, -0.13501102001039084,
        -0.08544127388224149, 0.03522629188210562,
)
_SYM4 = (
        0.03222310060407815, -0.01260396726226383, -0.09921954357695636, 0.29785779560553225,
        0.80373875180591614, 0.49761866763256292, -0.02963552764596039, -0.07576571478935668,
)
_SYM5 = (
        0.027333068345078, 0.029519490925775, -0.039134249302383, 0.199397533977394,
        0.723407690402421, 0.633978963458212, 0.016602105764522, -0.175328089908450,
        -0.021101834024759, 0.019538882735287,
)
_SYM6 = (
        0.015404109327027, 0.003490712084466, -0.117990111148191, -0.048311742585633,
        0.491055941926747, 0.787641141030194, 0.337929421727622, -0.072637522786462,
        -0.021060292512300, 0.044724901770665, 0.001767711864087, -0.007800708325034,
)
_SYM7 = (
        0.002681814568258, -0.001047384889692, -0.012636303403216, 0.030515513162982,
        0.067892693501372, -0.049552834937127, 0.017441255086855, 0.536101917091769,
        0.767764317003164, 0.288629631751927, -0.140047240442652, -0.107808237703821,
        0.004010244871534, 0.010268176708511,
)
_SYM8 = (
        -0.003382415951359, -0.000542132331635, 0.031695087810979, 0.007607487324918,
        -0.143294238350810, -0.061273359067938, 0.481359651258372, 0.777185751700574,
        0.364441894835509, -0.051945838107658, -0.027219029168752, 0.049137179673713,
        0.003808752013903, -0.014952258336792, -0.000302920514551, 0.001889950332768,
)
_SYM10 = (
        0.0007701598091030, 0.0000956388665879, -0.0086412992770191, -0.0014653825833081,
        0.0459272392237083, 0.0116098939129599, -0.1594942788488777, -0.0708805358733626,
        0.4716906668263991, 0.7695100370211090, 0.3838267612696101, -0.0355367403034847,
        -0.0319900568798241, 0.0499949720772958, 0.0057649120335782, -0.0203549398039241,
        -0.0008043589320530, 0.0045931735836929, -0.0000570360843902, -0.0004593294205334,
)
_COIF1 = (
        -0.0156557281354645, -0.0727326195128561, 0.3848648468642029, 0.8525720202122554,
        0.3378976624578092, -0.0727326195128561,
)
_COIF2 = (
        -0.0007205494453645, -0.0018232088709132, 0.0056211431711065, 0.0235962077162017,
        -0.0594274367855454, -0.0764421423447531, 0.4170051844216925, 0.8127236354455423,
        0.3861100668250532, -0.0673725547219630, -0.0414649367817581, 0.0164064277978058,
)
_COIF3 = (
        -0.0000345997728362, -0.0000709833031381, 0.0004662169601129, 0.0011175187708906,
        -0.0025745176887502, -0.0090079761366615, 0.0158805448636158, 0.0345550275730615,
        -0.0823019271068856, -0.0717998216193117, 0.4284834763776168, 0.7937772226256169,
        0.4051769024096150, -0.0611233900026726, -0.0657719112818552, 0.0234526961418362,
        0.0077825964273254, -0.0037935128644910,
)
_COIF4 = (
        -0.0000017849850031, -0.0000032596802369, 0.0000312298758654, 0.0000623390344610,
        -0.0002599745524878, -0.0005890207562444, 0.0012665619292991, 0.0037514361572790,
        -0.0056582866866115, -0.0152117315279485, 0.0250822618448678, 0.0393344271233433,
        -0.0962204420340021, -0.0666274742634348, 0.4343860564915321, 0.7822389309206135,
        0.4153084070304910, -0.0560773133167630, -0.0812666996808907, 0.0266823001560570,
        0.0160689439647787, -0.0073461663276432, -0.0016294920126020, 0.0008923136685824,
)
_COIF5 = (
        -0.0000000960401011, -0.0000001623799517, 0.0000020612203986, 0.0000037007277113,
        -0.0000212702216725, -0.0000412198619243, 0.0001403563281237, 0.0003018579416682,
        -0.0006375589261259, -0.0016616273039299, 0.0024315754425383, 0.0067615202206204,
        -0.0091595073386762, -0.0197583916009655, 0.0326747994670574, 0.0412875304721178,
        -0.1055631513073372, -0.0620377515749820, 0.4379823066591634, 0.7742936228603274,
        0.4215712667307543, -0.0520466702535548, -0.0919215880600861, 0.0281697442705324,
        0.0234083221189278, -0.0101315848469003, -0.0041593126275786, 0.0021782943778457,
        0.0003585777411618, -0.0002120818620675,
)


class Wavelet:
    """A discrete orthogonal wavelet (lowPassDecomposition / highPassDecomposition / reconstruction)."""

    def __init__(self, name: str, low: Tuple[float, ...], wavelet_id: int = WID_OTHER,
                 high: Tuple[float, ...] | None = None, vanishing_moments: int = 0):
        self._name = name
        self._low = tuple(float(v) for v in low)
        if high is None:
            L = len(self._low)
            high = tuple((1 if i % 2 == 0 else -1) * self._low[L - 1 - i] for i in range(L))
        self._high = tuple(float(v) for v in high)
        self.wavelet_id = wavelet_id
        self._vm = vanishing_moments

    def name(self) -> str:
        return self._name

    def lowPassDecomposition(self):
        return list(self._low)

    def highPassDecomposition(self):
        return list(self._high)

    def lowPassReconstruction(self):
        return list(self._low)

    def highPassReconstruction(self):
        return list(self._high)

    def vanishingMoments(self) -> int:
        return self._vm

    @property
    def filter_length(self) -> int:
        return len(self._low)

    def __repr__(self) -> str:
        return f"Wavelet({self._name}, L={len(self._low)})"


class Haar(Wavelet):
    """core/api/Haar.java: h = {1/sqrt2, 1/sqrt2}, g = {1/sqrt2, -1/sqrt2}."""

    INSTANCE: "Haar"

    def __init__(self):
        super().__init__("Haar", (_SQRT2_INV, _SQRT2_INV), WID_HAAR, (_SQRT2_INV, -_SQRT2_INV), 1)


Haar.INSTANCE = Haar()


class Daubechies:
    DB2 = Wavelet("db2", _DB2, WID_DB2, vanishing_moments=2)
    DB4 = Wavelet("db4", _DB4, WID_DB4, vanishing_moments=4)
    DB6 = Wavelet("db6", _DB6, WID_DB6, vanishing_moments=6)
    DB8 = Wavelet("db8", _DB8, WID_DB8, vanishing_moments=8)
    DB10 = Wavelet("db10", _DB10, WID_DB10, vanishing_moments=10)


class Symlet:
    SYM2 = Wavelet("sym2", _SYM2, vanishing_moments=2)
    SYM3 = Wavelet("sym3", _SYM3, vanishing_moments=3)
    SYM4 = Wavelet("sym4", _SYM4, WID_SYM4, vanishing_moments=4)
    SYM5 = Wavelet("sym5", _SYM5, vanishing_moments=5)
    SYM6 = Wavelet("sym6", _SYM6, vanishing_moments=6)
    SYM7 = Wavelet("sym7", _SYM7, vanishing_moments=7)
    SYM8 = Wavelet("sym8", _SYM8, WID_SYM8, vanishing_moments=8)
    SYM10 = Wavelet("sym10", _SYM10, vanishing_moments=10)


class Coiflet:
    COIF1 = Wavelet("coif1", _COIF1, WID_COIF1, vanishing_moments=2)
    COIF2 = Wavelet("coif2", _COIF2, WID_COIF2, vanishing_moments=4)
    COIF3 = Wavelet("coif3", _COIF3, WID_COIF3, vanishing_moments=6)
    COIF4 = Wavelet("coif4", _COIF4, vanishing_moments=8)
    COIF5 = Wavelet("coif5", _COIF5, WID_COIF5, vanishing_moments=10)


_REGISTRY: Dict[str, Wavelet] = {"haar": Haar.INSTANCE}
for _cls in (Daubechies, Symlet, Coiflet):
    for _k, _v in vars(_cls).items():
        if isinstance(_v, Wavelet):
            _REGISTRY[_k.lower()] = _v


def get_wavelet(name: str) -> Wavelet:
    """WaveletRegistry.getWavelet-style lookup by lower-case name ('haar', 'db4', 'sym8', 'coif5', ...)."""
    try:
        return _REGISTRY[name.lower()]
    except KeyError:
        raise KeyError(f"unknown wavelet {name!r}; known: {sorted(_REGISTRY)}") from None


def available_wavelets():
    return sorted(_REGISTRY)
