"""pyspark.ml.param-compatible Params system (Param, Params, TypeConverters).

Kept exactly as the reference API expects (mllib_multilayer_perceptron_classifier.py:35 builds
the estimator from keyword params): defaults vs user-set values, ``explainParams``, ``copy``,
``extractParamMap``, getters/setters, and JSON persistence of both maps.
"""
import copy as _copy
import uuid
import zlib


class TypeConverters:
    @staticmethod
    def identity(v):
        return v

    @staticmethod
    def toInt(v):
        if isinstance(v, bool) or int(v) != v:
            raise TypeError(f"Could not convert {v!r} to int")
        return int(v)

    @staticmethod
    def toFloat(v):
        return float(v)

    @staticmethod
    def toString(v):
        if not isinstance(v, str):
            raise TypeError(f"Could not convert {v!r} to string")
        return v

    @staticmethod
    def toBoolean(v):
        if not isinstance(v, bool):
            raise TypeError(f"Could not convert {v!r} to boolean")
        return v

    @staticmethod
    def toListInt(v):
        return [TypeConverters.toInt(x) for x in v]

    @staticmethod
    def toListFloat(v):
        return [float(x) for x in v]

    @staticmethod
    def toVector(v):
        from .linalg import DenseVector, Vector
        return v if isinstance(v, Vector) else DenseVector(v)


class Param:
    def __init__(self, parent, name, doc, typeConverter=None):
        self.parent = parent if isinstance(parent, str) else getattr(parent, "uid", "undefined")
        self.name = name
        self.doc = doc
        self.typeConverter = typeConverter or TypeConverters.identity

    def __repr__(self):
        return f"{self.parent}__{self.name}"

    def __hash__(self):
        return hash(str(self))

    def __eq__(self, other):
        return isinstance(other, Param) and self.parent == other.parent and self.name == other.name


def stable_hash(s: str) -> int:
    """Deterministic stand-in for pyspark's HasSeed default (which uses Python's randomised str hash)."""
    return zlib.crc32(s.encode()) & 0x7FFFFFFF


class Params:
    def __init__(self):
        self.uid = f"{type(self).__name__}_{uuid.uuid4().hex[-12:]}"
        self._paramMap = {}
        self._defaultParamMap = {}
        self._params = None
        for name in dir(type(self)):
            attr = getattr(type(self), name, None)
            if isinstance(attr, Param):
                p = Param(self.uid, attr.name, attr.doc, attr.typeConverter)
                setattr(self, name, p)

    @property
    def params(self):
        if self._params is None:
            self._params = sorted([getattr(self, n) for n in dir(self)
                                   if not n.startswith("__") and n != "params" and isinstance(getattr(self, n, None), Param)],
                                  key=lambda p: p.name)
        return self._params

    def getParam(self, name):
        p = getattr(self, name, None)
        if not isinstance(p, Param):
            raise ValueError(f"Cannot find param with name {name}")
        return p

    def hasParam(self, name):
        return isinstance(getattr(self, name, None), Param)

    def _resolve(self, param):
        return self.getParam(param) if isinstance(param, str) else param

    def isSet(self, param):
        return self._resolve(param) in self._paramMap

    def hasDefault(self, param):
        return self._resolve(param) in self._defaultParamMap

    def isDefined(self, param):
        return self.isSet(param) or self.hasDefault(param)

    def getOrDefault(self, param):
        p = self._resolve(param)
        if p in self._paramMap:
            return self._paramMap[p]
        if p in self._defaultParamMap:
            return self._defaultParamMap[p]
        raise KeyError(f"Param {p.name} is not set and has no default")

    def _set(self, **kwargs):
        for k, v in kwargs.items():
            p = self.getParam(k)
            if v is not None:
                v = p.typeConverter(v)
            self._paramMap[p] = v
        return self

    def set(self, param, value):
        self._paramMap[self._resolve(param)] = value
        return self

    def _setDefault(self, **kwargs):
        for k, v in kwargs.items():
            p = self.getParam(k)
            if v is not None and not callable(v):
                v = p.typeConverter(v)
            self._defaultParamMap[p] = v
        return self

    def clear(self, param):
        self._paramMap.pop(self._resolve(param), None)

    def explainParam(self, param):
        p = self._resolve(param)
        vals = []
        if self.hasDefault(p):
            vals.append(f"default: {self._defaultParamMap[p]}")
        if self.isSet(p):
            vals.append(f"current: {self._paramMap[p]}")
        return f"{p.name}: {p.doc} ({', '.join(vals) if vals else 'undefined'})"

    def explainParams(self):
        return "\n".join(self.explainParam(p) for p in self.params)

    def extractParamMap(self, extra=None):
        m = dict(self._defaultParamMap)
        m.update(self._paramMap)
        if extra:
            m.update(extra)
        return m

    def copy(self, extra=None):
        that = _copy.copy(self)
        that._paramMap = dict(self._paramMap)
        that._defaultParamMap = dict(self._defaultParamMap)
        if extra:
            for p, v in extra.items():
                that._paramMap[that.getParam(p.name)] = v
        return that

    def _copyValues(self, to, extra=None):
        pm = self.extractParamMap(extra)
        for p, v in pm.items():
            if to.hasParam(p.name):
                if p in self._paramMap or (extra and p in extra):
                    to._paramMap[to.getParam(p.name)] = v
                else:
                    to._defaultParamMap[to.getParam(p.name)] = v
        return to

    def _param_json(self, which):
        from .linalg import Vector
        src = self._paramMap if which == "set" else self._defaultParamMap
        out = {}
        for p, v in src.items():
            if isinstance(v, Vector):
                v = {"type": 1, "values": v.toArray().tolist()}
            out[p.name] = v
        return out


# ---- shared param mixins (pyspark.ml.param.shared) --------------------------------------
def _mixin(name, pname, doc, conv, default=None, has_default=True):
    def getter(self):
        return self.getOrDefault(getattr(self, pname))

    def setter(self, value):
        return self._set(**{pname: value})

    attrs = {pname: Param("undefined", pname, doc, conv),
             "get" + pname[0].upper() + pname[1:]: getter,
             "set" + pname[0].upper() + pname[1:]: setter}
    cls = type(name, (Params,), attrs)
    cls._mixin_default = (pname, default, has_default)
    return cls


HasFeaturesCol = _mixin("HasFeaturesCol", "featuresCol", "features column name.", TypeConverters.toString, "features")
HasLabelCol = _mixin("HasLabelCol", "labelCol", "label column name.", TypeConverters.toString, "label")
HasPredictionCol = _mixin("HasPredictionCol", "predictionCol", "prediction column name.", TypeConverters.toString,
                          "prediction")
HasProbabilityCol = _mixin("HasProbabilityCol", "probabilityCol", "Column name for predicted class conditional "
                           "probabilities.", TypeConverters.toString, "probability")
HasRawPredictionCol = _mixin("HasRawPredictionCol", "rawPredictionCol", "raw prediction (a.k.a. confidence) column "
                             "name.", TypeConverters.toString, "rawPrediction")
HasMaxIter = _mixin("HasMaxIter", "maxIter", "max number of iterations (>= 0).", TypeConverters.toInt, 100)
HasTol = _mixin("HasTol", "tol", "the convergence tolerance for iterative algorithms (>= 0).",
                TypeConverters.toFloat, 1e-6)
HasStepSize = _mixin("HasStepSize", "stepSize", "Step size to be used for each iteration of optimization (>= 0).",
                     TypeConverters.toFloat, 0.03)
HasSeed = _mixin("HasSeed", "seed", "random seed.", TypeConverters.toInt, None)
HasSolver = _mixin("HasSolver", "solver", "The solver algorithm for optimization.", TypeConverters.toString, "l-bfgs")
HasBlockSize = _mixin("HasBlockSize", "blockSize", "block size for stacking input data in matrices.",
                      TypeConverters.toInt, 128)
HasWeightCol = _mixin("HasWeightCol", "weightCol", "weight column name.", TypeConverters.toString, None, False)
HasThresholds = _mixin("HasThresholds", "thresholds", "Thresholds in multi-class classification.",
                       TypeConverters.toListFloat, None, False)


def apply_mixin_defaults(obj):
    for klass in type(obj).__mro__:
        d = klass.__dict__.get("_mixin_default")
        if d:
            pname, default, has_default = d
            if has_default and not obj.hasDefault(pname):
                if pname == "seed":
                    default = stable_hash(type(obj).__name__)
                obj._setDefault(**{pname: default})
