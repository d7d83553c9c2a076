"""Core Python API: :class:`Dataset` and :class:`Booster` over the native C API.

Mirrors the user-facing surface of the reference python package
(python-package/lightgbm/basic.py: Dataset, Booster, LightGBMError) so user
code can switch by changing the import. Data flows to the native library
through ctypes without copies where the input is already contiguous.
"""
from __future__ import annotations

import ctypes
import warnings
import json
import os
from copy import deepcopy
from pathlib import Path
from typing import Set, Any, Callable, Dict, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np

from .libpath import find_lib_path

try:  # optional inputs
    import pandas as pd  # type: ignore
except Exception:  # pragma: no cover
    pd = None
try:
    import scipy.sparse as sp  # type: ignore
except Exception:  # pragma: no cover
    sp = None

__all__ = ["LightGBMError", "Dataset", "Booster", "Sequence", "register_logger", "device_count", "phase_timer_report"]

C_API_DTYPE_FLOAT32 = 0
C_API_DTYPE_FLOAT64 = 1
C_API_DTYPE_INT32 = 2
C_API_DTYPE_INT64 = 3
C_API_PREDICT_NORMAL = 0
C_API_PREDICT_RAW_SCORE = 1
C_API_PREDICT_LEAF_INDEX = 2
C_API_PREDICT_CONTRIB = 3
C_API_FEATURE_IMPORTANCE_SPLIT = 0
C_API_FEATURE_IMPORTANCE_GAIN = 1

_FIELD_TYPES = {"label": np.float32, "weight": np.float32, "init_score": np.float64, "group": np.int32,
                "position": np.int32}


class LightGBMError(Exception):
    """Error raised by the native library."""


def _load_lib() -> ctypes.CDLL:
    lib = ctypes.cdll.LoadLibrary(find_lib_path())
    lib.LGBM_GetLastError.restype = ctypes.c_char_p
    return lib


_LIB = _load_lib()
_LOG_CALLBACK = None
_LOGGER: Any = None


def _check(ret: int) -> None:
    if ret != 0:
        raise LightGBMError(_LIB.LGBM_GetLastError().decode("utf-8"))


def _c_str(s: str) -> ctypes.c_char_p:
    return ctypes.c_char_p(s.encode("utf-8"))


def _log_info(msg: str) -> None:
    if _LOGGER is not None:
        _LOGGER.info(msg)
    else:
        print(msg, flush=True)


def _log_warning(msg: str) -> None:
    """Python-side warnings: the registered logger's warning method, else ``warnings.warn``
    (reference basic.py _DummyLogger / _log_warning)."""
    if _LOGGER is not None:
        _LOGGER.warning(msg)
    else:
        warnings.warn(msg, stacklevel=3)


def _log_sink(msg: bytes) -> None:
    text = msg.decode("utf-8").rstrip("\n")
    if not text:
        return
    _log_info(text)


def register_logger(logger: Any, info_method_name: str = "info", warning_method_name: str = "warning") -> None:
    """Route native log lines (``info_method_name``) and Python-side warnings
    (``warning_method_name``) to a logger object."""
    global _LOGGER
    for name in (info_method_name, warning_method_name):
        if not callable(getattr(logger, name, None)):
            raise TypeError(f"Logger must provide '{info_method_name}' and '{warning_method_name}' method")

    class _Wrap:
        def info(self, m):
            getattr(logger, info_method_name)(m)

        def warning(self, m):
            getattr(logger, warning_method_name)(m)

    _LOGGER = _Wrap()


def _install_log_callback() -> None:
    global _LOG_CALLBACK
    cb_type = ctypes.CFUNCTYPE(None, ctypes.c_char_p)
    _LOG_CALLBACK = cb_type(_log_sink)
    _check(_LIB.LGBM_RegisterLogCallback(_LOG_CALLBACK))


_install_log_callback()


def device_count() -> int:
    """Number of visible gfx950 GPUs (0 when none)."""
    out = ctypes.c_int(0)
    _check(_LIB.LGBM_DeviceCount(ctypes.byref(out)))
    return out.value


def phase_timer_report() -> str:
    """Per-phase timing report (populated when LGAP_TIMETAG=1)."""
    return _get_string(lambda n, ol, buf: _LIB.LGBM_PhaseTimerReport(ctypes.c_int64(n), ol, buf))


def _get_string(fn: Callable, size: int = 1 << 16) -> str:
    out_len = ctypes.c_int64(0)
    buf = ctypes.create_string_buffer(size)
    _check(fn(size, ctypes.byref(out_len), buf))
    if out_len.value > size:
        size = out_len.value
        buf = ctypes.create_string_buffer(size)
        _check(fn(size, ctypes.byref(out_len), buf))
    return buf.value.decode("utf-8")


def _param_value(v: Any) -> str:
    if isinstance(v, (list, tuple, np.ndarray)):
        if len(v) and isinstance(v[0], (list, tuple, np.ndarray)):
            # list of lists (interaction_constraints): "[0,1,2],[3,4]"
            return ",".join("[" + ",".join(_param_value(x) for x in inner) + "]" for inner in v)
        return ",".join(_param_value(x) for x in v)
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return repr(v)
    return str(v)


def param_dict_to_str(params: Optional[Dict[str, Any]]) -> str:
    if not params:
        return ""
    pairs = []
    for k, v in params.items():
        if v is None or callable(v):
            continue
        if isinstance(v, dict):
            continue
        if isinstance(v, (list, tuple)) and len(v) == 0:
            continue
        pairs.append(f"{k}={_param_value(v)}")
    return " ".join(pairs)


def dump_param_aliases() -> Dict[str, List[str]]:
    return json.loads(_get_string(lambda n, ol, buf: _LIB.LGBM_DumpParamAliases(ctypes.c_int64(n), ol, buf)))


_ALIASES: Optional[Dict[str, List[str]]] = None


def _aliases() -> Dict[str, List[str]]:
    global _ALIASES
    if _ALIASES is None:
        _ALIASES = dump_param_aliases()
    return _ALIASES


class _ConfigAliases:
    """Parameter alias lookup (reference basic.py ``_ConfigAliases``), backed by the native
    parameter table (``LGBM_DumpParamAliases``)."""

    @staticmethod
    def get(*args: str) -> Set[str]:
        out: Set[str] = set()
        for name in args:
            out.add(name)
            out.update(_aliases().get(name, []))
        return out

    @staticmethod
    def get_sorted(name: str) -> List[str]:
        return [name] + [a for a in _aliases().get(name, []) if a != name]

    @staticmethod
    def get_by_alias(*args: str) -> Set[str]:
        out: Set[str] = set(args)
        for arg in args:
            for main, al in _aliases().items():
                if arg == main or arg in al:
                    out.add(main)
                    out.update(al)
        return out


def _choose_param_value(main: str, params: Dict[str, Any], default: Any) -> Dict[str, Any]:
    """Collapse all aliases of `main` into `main` (first found wins)."""
    params = dict(params)
    names = [main] + [a for a in _aliases().get(main, []) if a != main]
    found = None
    for n in names:
        if n in params:
            if found is None:
                found = params[n]
            params.pop(n)
    params[main] = default if found is None else found
    return params


def _to_float_matrix(data: Any) -> Tuple[np.ndarray, int]:
    arr = np.asarray(data)
    if arr.ndim != 2:
        raise ValueError("Input numpy.ndarray or list must be 2 dimensional")
    if arr.dtype == np.float32:
        return np.ascontiguousarray(arr), C_API_DTYPE_FLOAT32
    return np.ascontiguousarray(arr, dtype=np.float64), C_API_DTYPE_FLOAT64


def _pandas_to_numpy(df: Any, categorical_feature: Any, pandas_categorical: Optional[List[List[Any]]]):
    """Convert a DataFrame, mapping category columns to their codes."""
    cat_cols = [c for c in df.columns if str(df[c].dtype) == "category"]
    if pandas_categorical is None:
        pandas_categorical = [list(df[c].cat.categories) for c in cat_cols]
    else:
        if len(cat_cols) != len(pandas_categorical):
            raise ValueError("train and valid dataset categorical_feature do not match.")
    ordered = [bool(df[c].cat.ordered) for c in cat_cols]
    df = df.copy() if cat_cols else df
    for col, cats in zip(cat_cols, pandas_categorical):
        if list(df[col].cat.categories) != list(cats):
            df[col] = df[col].cat.set_categories(cats)
        df[col] = df[col].cat.codes.replace({-1: np.nan}).astype(np.float64)
    feature_names = [str(c) for c in df.columns]
    if categorical_feature == "auto":
        # unordered category columns only (reference basic.py _data_from_pandas); an explicit
        # list is taken as given
        categorical_feature = [str(c) for c, o in zip(cat_cols, ordered) if not o]
    values = df.to_numpy(dtype=np.float64, na_value=np.nan) if hasattr(df, "to_numpy") else df.values.astype(np.float64)
    return values, feature_names, categorical_feature, pandas_categorical


def _is_sparse(x: Any) -> bool:
    return sp is not None and sp.issparse(x)


class _ArrowSchema(ctypes.Structure):
    _fields_ = [("format", ctypes.c_char_p), ("name", ctypes.c_char_p), ("metadata", ctypes.c_char_p),
                ("flags", ctypes.c_int64), ("n_children", ctypes.c_int64), ("children", ctypes.c_void_p),
                ("dictionary", ctypes.c_void_p), ("release", ctypes.c_void_p), ("private_data", ctypes.c_void_p)]


class _ArrowArray(ctypes.Structure):
    _fields_ = [("length", ctypes.c_int64), ("null_count", ctypes.c_int64), ("offset", ctypes.c_int64),
                ("n_buffers", ctypes.c_int64), ("n_children", ctypes.c_int64), ("buffers", ctypes.c_void_p),
                ("children", ctypes.c_void_p), ("dictionary", ctypes.c_void_p), ("release", ctypes.c_void_p),
                ("private_data", ctypes.c_void_p)]


_ARROW_RELEASE = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


def _is_arrow(x: Any) -> bool:
    mod = type(x).__module__ or ""
    if not mod.startswith("pyarrow"):
        return False
    import pyarrow as pa

    return isinstance(x, (pa.Table, pa.RecordBatch, pa.Array, pa.ChunkedArray))


class _ArrowExport:
    """Exports a pyarrow Table / RecordBatch / (Chunked)Array through the Arrow C data
    interface for the native reader (lgap/arrow.h); releases the exported structs on exit."""

    def __init__(self, obj: Any) -> None:
        import pyarrow as pa

        if isinstance(obj, pa.Table):
            parts, schema_src = obj.to_batches(), obj.schema
        elif isinstance(obj, pa.RecordBatch):
            parts, schema_src = [obj], obj.schema
        elif isinstance(obj, pa.ChunkedArray):
            parts, schema_src = list(obj.chunks), obj.type
        elif isinstance(obj, pa.Array):
            parts, schema_src = [obj], obj.type
        else:
            raise TypeError(f"Unsupported Arrow object {type(obj).__name__}")
        self.n = len(parts)
        self.chunks = (_ArrowArray * max(1, self.n))()
        self.schema = _ArrowSchema()
        schema_src._export_to_c(ctypes.addressof(self.schema))
        for i, part in enumerate(parts):
            tmp = _ArrowSchema()
            part._export_to_c(ctypes.addressof(self.chunks[i]), ctypes.addressof(tmp))
            _ArrowExport._release(tmp)

    @staticmethod
    def _release(struct: ctypes.Structure) -> None:
        if struct.release:
            _ARROW_RELEASE(struct.release)(ctypes.addressof(struct))

    def __enter__(self) -> "_ArrowExport":
        return self

    def __exit__(self, *exc: Any) -> None:
        for i in range(self.n):
            _ArrowExport._release(self.chunks[i])
        _ArrowExport._release(self.schema)


def _is_pandas(x: Any) -> bool:
    return pd is not None and isinstance(x, pd.DataFrame)


def _is_path(x: Any) -> bool:
    return isinstance(x, (str, Path))


class Sequence:
    """Generic row-access data source (``__getitem__`` + ``__len__``), consumed in batches."""

    batch_size = 4096

    def __getitem__(self, idx):  # pragma: no cover - interface
        raise NotImplementedError

    def __len__(self):  # pragma: no cover - interface
        raise NotImplementedError


class Dataset:
    """Training / validation data, binned lazily on first use.

    Reference: python-package/lightgbm/basic.py Dataset (constructor
    arguments, lazy ``construct``, ``create_valid``, field setters).
    """

    def __init__(self, data: Any, label: Any = None, reference: Optional["Dataset"] = None, weight: Any = None,
                 group: Any = None, init_score: Any = None, feature_name: Any = "auto",
                 categorical_feature: Any = "auto", params: Optional[Dict[str, Any]] = None,
                 free_raw_data: bool = True, position: Any = None):
        self.handle: Optional[ctypes.c_void_p] = None
        self.data = data
        self.label = label
        self.reference = reference
        self.weight = weight
        self.group = group
        self.init_score = init_score
        self.position = position
        self.feature_name = feature_name
        self.categorical_feature = categorical_feature
        self.params = deepcopy(params) if params else {}
        self.free_raw_data = free_raw_data
        self.used_indices: Optional[np.ndarray] = None
        self._predictor = None
        self.pandas_categorical: Optional[List[List[Any]]] = None
        self._params_back_up = None
        self.version = 0

    # ------------------------------------------------------------------ construction
    def __del__(self):
        try:
            self._free_handle()
        except Exception:
            pass

    def _free_handle(self) -> "Dataset":
        if self.handle is not None:
            _check(_LIB.LGBM_DatasetFree(self.handle))
            self.handle = None
        return self

    def construct(self) -> "Dataset":
        if self.handle is not None:
            return self
        if self.reference is not None:
            self.reference.construct()
            # a validation set / subset is binned like its reference (reference basic.py construct)
            ref_params, own = self.reference.get_params(), self.get_params()
            if own != ref_params:
                cat_keys = {"categorical_feature"} | set(_aliases().get("categorical_feature", []))
                strip = lambda d: {k: v for k, v in d.items() if k not in cat_keys}  # noqa: E731
                if strip(own) != strip(ref_params):
                    _log_warning("Overriding the parameters from Reference Dataset.")
                self._update_params(ref_params)
        if self.used_indices is not None and self.reference is not None:
            # subset of a constructed dataset
            idx = np.ascontiguousarray(self.used_indices, dtype=np.int32)
            out = ctypes.c_void_p()
            _check(_LIB.LGBM_DatasetGetSubset(self.reference.handle, idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                              ctypes.c_int32(idx.size), _c_str(param_dict_to_str(self.params)),
                                              ctypes.byref(out)))
            self.handle = out
            # the native subset inherits the reference's init score; a different model needs
            # the reference's raw rows
            if self._predictor is not None and self._predictor is not self.reference._predictor:
                if self.reference.data is None:
                    raise LightGBMError("Cannot set predictor after freed raw data, "
                                        "set free_raw_data=False when construct Dataset to avoid this.")
                self.init_score = self._init_score_from_predictor(self._predictor, self.reference.data,
                                                                  self.used_indices)
            self._set_metadata()
            # reference basic.py construct: a kept subset materialises its rows and label
            if not self.free_raw_data and self.reference.data is not None:
                self.get_data()
            if self.get_label() is None:
                raise ValueError("Label should not be None.")
            return self
        if self._predictor is not None:  # the continued model's scores replace any init_score
            self.init_score = self._init_score_from_predictor(self._predictor, self.data)
        self._lazy_init(self.data)
        return self

    def _build_params(self, categorical_indices: List[int]) -> str:
        # the resolved categorical columns become a Dataset parameter (categorical_column), which
        # the Booster inherits and the model text records (reference basic.py Dataset._lazy_init)
        if categorical_indices:
            want = sorted(set(categorical_indices))
            for alias in ["categorical_feature"] + _aliases().get("categorical_feature", []):
                if alias in self.params:
                    cur = self.params[alias]
                    if not (isinstance(cur, list) and set(cur) == set(want)):
                        _log_warning(f"{alias} in param dict is overridden.")
                    self.params.pop(alias, None)
            self.params["categorical_column"] = want
        return param_dict_to_str(self.params)

    def _resolve_categorical(self, feature_names: Optional[List[str]], ncol: int) -> List[int]:
        # a DataFrame's "auto" resolves to its unordered category columns without changing the
        # user-facing categorical_feature (reference basic.py _lazy_init)
        cf = getattr(self, "_frame_categorical", None)
        if cf is None:
            cf = self.categorical_feature
        if cf is None or cf == "auto" or (isinstance(cf, (list, tuple)) and len(cf) == 0):
            return []
        out = []
        for c in cf:
            if isinstance(c, (int, np.integer)):
                out.append(int(c))
            elif feature_names is not None and c in feature_names:
                out.append(feature_names.index(c))
            else:
                raise ValueError(f"Could not find categorical_feature {c} in data")
        return sorted(set(out))

    def _lazy_init(self, data: Any) -> None:
        ref = self.reference.handle if self.reference is not None else None
        feature_names = None
        if _is_pandas(data):
            pc = self.reference.pandas_categorical if self.reference is not None else None
            data, feature_names, cat, self.pandas_categorical = _pandas_to_numpy(data, self.categorical_feature, pc)
            self._frame_categorical = cat
        elif self.reference is not None:
            self.pandas_categorical = self.reference.pandas_categorical
        if self.feature_name != "auto" and self.feature_name is not None:
            feature_names = list(self.feature_name)
        out = ctypes.c_void_p()
        if _is_arrow(data):
            names = list(data.schema.names) if hasattr(data, "schema") else None
            cat_idx = self._resolve_categorical(feature_names or names, len(names or []))
            with _ArrowExport(data) as ex:
                _check(_LIB.LGBM_DatasetCreateFromArrow(ctypes.c_int64(ex.n), ex.chunks, ctypes.byref(ex.schema),
                                                        _c_str(self._build_params(cat_idx)), ref, ctypes.byref(out)))
        elif _is_path(data):
            cat_idx = self._resolve_categorical(feature_names, -1)
            _check(_LIB.LGBM_DatasetCreateFromFile(_c_str(str(data)), _c_str(self._build_params(cat_idx)), ref,
                                                   ctypes.byref(out)))
        elif _is_sparse(data):
            mat = data.tocsr() if data.format not in ("csr", "csc") else data
            cat_idx = self._resolve_categorical(feature_names, mat.shape[1])
            params = _c_str(self._build_params(cat_idx))
            if mat.format == "csr":
                indptr, ip_type = self._indptr(mat.indptr)
                vals, vtype = self._values(mat.data)
                indices = np.ascontiguousarray(mat.indices, dtype=np.int32)
                _check(_LIB.LGBM_DatasetCreateFromCSR(indptr.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(ip_type),
                                                      indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                      vals.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(vtype),
                                                      ctypes.c_int64(indptr.size), ctypes.c_int64(vals.size),
                                                      ctypes.c_int64(mat.shape[1]), params, ref, ctypes.byref(out)))
            else:
                colptr, ip_type = self._indptr(mat.indptr)
                vals, vtype = self._values(mat.data)
                indices = np.ascontiguousarray(mat.indices, dtype=np.int32)
                _check(_LIB.LGBM_DatasetCreateFromCSC(colptr.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(ip_type),
                                                      indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                      vals.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(vtype),
                                                      ctypes.c_int64(colptr.size), ctypes.c_int64(vals.size),
                                                      ctypes.c_int64(mat.shape[0]), params, ref, ctypes.byref(out)))
        elif isinstance(data, list) and data and isinstance(data[0], np.ndarray) and data[0].ndim == 2:
            mats = [_to_float_matrix(m)[0].astype(np.float64, copy=False) for m in data]
            ncol = mats[0].shape[1]
            cat_idx = self._resolve_categorical(feature_names, ncol)
            ptrs = (ctypes.c_void_p * len(mats))(*[m.ctypes.data_as(ctypes.c_void_p) for m in mats])
            nrows = np.array([m.shape[0] for m in mats], dtype=np.int32)
            _check(_LIB.LGBM_DatasetCreateFromMats(ctypes.c_int32(len(mats)), ptrs, ctypes.c_int(C_API_DTYPE_FLOAT64),
                                                   nrows.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                   ctypes.c_int32(ncol), ctypes.c_int(1),
                                                   _c_str(self._build_params(cat_idx)), ref, ctypes.byref(out)))
        elif isinstance(data, Sequence) or (isinstance(data, list) and data and isinstance(data[0], Sequence)):
            seqs = data if isinstance(data, list) else [data]
            rows = []
            for s in seqs:
                for i in range(0, len(s), s.batch_size):
                    rows.append(np.asarray(s[i:min(len(s), i + s.batch_size)], dtype=np.float64))
            mat = np.vstack(rows)
            self._lazy_init_mat(mat, feature_names, ref, out)
        else:
            if hasattr(data, "__array__") or isinstance(data, list):
                self._lazy_init_mat(np.asarray(data), feature_names, ref, out)
            else:
                raise TypeError(f"Cannot initialize Dataset from {type(data).__name__}")
        self.handle = out
        self._set_metadata()
        if feature_names is not None:
            self.set_feature_name(feature_names)
        if self.free_raw_data:
            self.data = None

    def _lazy_init_mat(self, arr: np.ndarray, feature_names, ref, out) -> None:
        mat, dtype = _to_float_matrix(arr)
        cat_idx = self._resolve_categorical(feature_names, mat.shape[1])
        _check(_LIB.LGBM_DatasetCreateFromMat(mat.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(dtype),
                                              ctypes.c_int32(mat.shape[0]), ctypes.c_int32(mat.shape[1]),
                                              ctypes.c_int(1), _c_str(self._build_params(cat_idx)), ref,
                                              ctypes.byref(out)))

    @staticmethod
    def _indptr(a: np.ndarray):
        if a.dtype == np.int32:
            return np.ascontiguousarray(a), C_API_DTYPE_INT32
        return np.ascontiguousarray(a, dtype=np.int64), C_API_DTYPE_INT64

    @staticmethod
    def _values(a: np.ndarray):
        if a.dtype == np.float32:
            return np.ascontiguousarray(a), C_API_DTYPE_FLOAT32
        return np.ascontiguousarray(a, dtype=np.float64), C_API_DTYPE_FLOAT64

    def _set_metadata(self) -> None:
        if self.label is not None:
            self.set_label(self.label)
        if self.weight is not None:
            self.set_weight(self.weight)
        if self.group is not None:
            self.set_group(self.group)
        if self.init_score is not None:
            self.set_init_score(self.init_score)
        if self.position is not None:
            self.set_position(self.position)

    def create_valid(self, data: Any, label: Any = None, weight: Any = None, group: Any = None,
                     init_score: Any = None, params: Optional[Dict[str, Any]] = None, position: Any = None) -> "Dataset":
        return Dataset(data, label=label, reference=self, weight=weight, group=group, init_score=init_score,
                       params=params if params is not None else self.params, free_raw_data=self.free_raw_data,
                       position=position, feature_name=self.feature_name, categorical_feature=self.categorical_feature)

    def subset(self, used_indices: Sequence[int], params: Optional[Dict[str, Any]] = None) -> "Dataset":
        ret = Dataset(None, reference=self, feature_name=self.feature_name, categorical_feature=self.categorical_feature,
                      params=params if params is not None else self.params, free_raw_data=self.free_raw_data)
        ret.used_indices = np.sort(np.asarray(used_indices, dtype=np.int32))
        ret.pandas_categorical = self.pandas_categorical
        ret._predictor = self._predictor
        return ret

    # ------------------------------------------------------------------ fields
    def set_field(self, field_name: str, data: Any) -> "Dataset":
        if self.handle is None:
            raise LightGBMError(f"Cannot set {field_name} before construct dataset")
        if data is None:
            _check(_LIB.LGBM_DatasetSetField(self.handle, _c_str(field_name), None, ctypes.c_int(0),
                                             ctypes.c_int(C_API_DTYPE_FLOAT32)))
            return self
        if _is_arrow(data):
            with _ArrowExport(data) as ex:
                _check(_LIB.LGBM_DatasetSetFieldFromArrow(self.handle, _c_str(field_name), ctypes.c_int64(ex.n),
                                                          ex.chunks, ctypes.byref(ex.schema)))
            self.version += 1
            return self
        dtype = _FIELD_TYPES.get(field_name, np.float32)
        if field_name == "init_score":
            arr = np.asarray(data, dtype=np.float64)
            if arr.ndim == 2:  # multiclass: store class-major
                arr = arr.T
            arr = np.ascontiguousarray(arr.ravel())
        else:
            arr = np.ascontiguousarray(np.asarray(data).ravel(), dtype=dtype)
        ctype = {np.float32: C_API_DTYPE_FLOAT32, np.float64: C_API_DTYPE_FLOAT64, np.int32: C_API_DTYPE_INT32}[
            arr.dtype.type]
        _check(_LIB.LGBM_DatasetSetField(self.handle, _c_str(field_name), arr.ctypes.data_as(ctypes.c_void_p),
                                         ctypes.c_int(arr.size), ctypes.c_int(ctype)))
        self.version += 1
        return self

    def get_field(self, field_name: str) -> Optional[np.ndarray]:
        if self.handle is None:
            raise LightGBMError(f"Cannot get {field_name} before construct Dataset")
        out_len = ctypes.c_int(0)
        out_ptr = ctypes.c_void_p()
        out_type = ctypes.c_int(0)
        _check(_LIB.LGBM_DatasetGetField(self.handle, _c_str(field_name), ctypes.byref(out_len), ctypes.byref(out_ptr),
                                         ctypes.byref(out_type)))
        if not out_ptr.value or out_len.value == 0:
            return None
        ct = {C_API_DTYPE_FLOAT32: ctypes.c_float, C_API_DTYPE_FLOAT64: ctypes.c_double,
              C_API_DTYPE_INT32: ctypes.c_int32}[out_type.value]
        arr = np.ctypeslib.as_array(ctypes.cast(out_ptr, ctypes.POINTER(ct)), shape=(out_len.value,)).copy()
        if field_name == "init_score":
            n = self.num_data()
            if n > 0 and arr.size > n and arr.size % n == 0:  # multiclass: stored class-major
                arr = arr.reshape(arr.size // n, n).T.copy()
        # "group" is returned as query boundaries (reference basic.py get_field); get_group()
        # gives the sizes
        return arr

    def set_label(self, label: Any) -> "Dataset":
        self.label = label
        if self.handle is not None and label is not None:
            if pd is not None and isinstance(label, (pd.Series, pd.DataFrame)):
                label = np.asarray(label).ravel()
            self.set_field("label", label)
            self.label = self.get_field("label")  # the stored (float32) values
        return self

    def set_weight(self, weight: Any) -> "Dataset":
        if weight is not None and np.all(np.asarray(weight) == 1):
            weight = None
        self.weight = weight
        if self.handle is not None and weight is not None:
            self.set_field("weight", weight)
            self.weight = self.get_field("weight")
        return self

    def set_init_score(self, init_score: Any) -> "Dataset":
        self.init_score = init_score
        if self.handle is not None and init_score is not None:
            self.set_field("init_score", init_score)
            self.init_score = self.get_field("init_score")
        return self

    def set_group(self, group: Any) -> "Dataset":
        self.group = group
        if self.handle is not None and group is not None:
            self.set_field("group", np.asarray(group, dtype=np.int32))
        return self

    def set_position(self, position: Any) -> "Dataset":
        self.position = position
        if self.handle is not None and position is not None:
            self.set_field("position", np.asarray(position, dtype=np.int32))
        return self

    def get_label(self):
        if self.label is None and self.handle is not None:
            self.label = self.get_field("label")
        return self.label

    def get_weight(self):
        if self.weight is None and self.handle is not None:
            self.weight = self.get_field("weight")
        return self.weight

    def get_init_score(self):
        if self.init_score is None and self.handle is not None:
            self.init_score = self.get_field("init_score")
        return self.init_score

    def get_group(self):
        if self.group is None and self.handle is not None:
            b = self.get_field("group")
            self.group = None if b is None else np.diff(b)
        return self.group

    def get_position(self):
        if self.position is None and self.handle is not None:
            self.position = self.get_field("position")
        return self.position

    def get_data(self):
        """The raw data of the Dataset; a subset slices its reference's raw data on first use
        (reference basic.py Dataset.get_data)."""
        if self.handle is None:
            raise Exception("Cannot get data before construct Dataset")
        if self.used_indices is not None and self.reference is not None and not getattr(self, "_sliced", False):
            self.data = self.reference.data
            if self.data is not None:
                if isinstance(self.data, np.ndarray) or _is_sparse(self.data):
                    self.data = self.data[self.used_indices, :]
                elif _is_pandas(self.data):
                    self.data = self.data.iloc[self.used_indices].copy()
                elif isinstance(self.data, Sequence):
                    self.data = self.data[self.used_indices]
                elif _is_arrow(self.data):
                    self.data = self.data.take(self.used_indices)
                elif not _is_path(self.data):
                    _log_warning(f"Cannot subset {type(self.data).__name__} type of raw data.\n"
                                 "Returning original raw data")
            self._sliced = True
        if self.data is None:
            raise LightGBMError("Cannot call `get_data` after freed raw data, "
                                "set free_raw_data=False when construct Dataset to avoid this.")
        return self.data

    _DATASET_PARAMS = ("bin_construct_sample_cnt", "categorical_feature", "data_random_seed", "enable_bundle",
                       "feature_pre_filter", "forcedbins_filename", "group_column", "header", "ignore_column",
                       "is_enable_sparse", "label_column", "linear_tree", "max_bin", "max_bin_by_feature",
                       "min_data_in_bin", "pre_partition", "precise_float_parser", "two_round", "use_missing",
                       "weight_column", "zero_as_missing")

    def get_params(self) -> Dict[str, Any]:
        """The Dataset-level parameters among ``params`` (binning / loading; aliases included),
        reference basic.py Dataset.get_params."""
        if not self.params:
            return {}
        names = set()
        for k in self._DATASET_PARAMS:
            names.add(k)
            names.update(_aliases().get(k, []))
        return {k: v for k, v in self.params.items() if k in names}

    def set_reference(self, reference: "Dataset") -> "Dataset":
        self.reference = reference
        # a validation set continues from the same model as its training set
        if reference is not None and reference._predictor is not None:
            self._set_predictor(reference._predictor)
        return self

    # ------------------------------------------------------------------ continued training
    def _init_score_from_predictor(self, predictor: "Booster", data: Any,
                                   used_indices: Optional[np.ndarray] = None) -> Optional[np.ndarray]:
        """Raw scores of ``predictor`` on ``data`` (array / frame / sparse / file path), restricted to
        ``used_indices`` for a subset (reference basic.py ``_set_init_score_by_predictor``)."""
        if data is None:
            return None
        if _is_path(data):
            header = str(self.params.get("header", self.params.get("has_header", False))).lower() in ("true", "1")
            raw = predictor.predict(str(data), raw_score=True, data_has_header=header)
        else:
            raw = predictor.predict(data, raw_score=True)
        raw = np.asarray(raw, dtype=np.float64)
        if used_indices is not None:
            raw = raw[np.asarray(used_indices, dtype=np.int64)]
        return raw

    def _set_predictor(self, predictor: Optional["Booster"]) -> "Dataset":
        """Attach the model training continues from; its raw scores become this Dataset's init
        score (now when constructed, else at construction). Reference: basic.py ``_set_predictor``."""
        if predictor is self._predictor:
            return self
        self._predictor = predictor
        if predictor is None or self.handle is None:
            return self  # construct() applies it
        if self.data is not None:
            self.set_init_score(self._init_score_from_predictor(predictor, self.data))
        elif self.used_indices is not None and self.reference is not None and self.reference._predictor is predictor:
            pass  # inherited from the reference at subset construction
        elif self.used_indices is not None and self.reference is not None and self.reference.data is not None:
            self.set_init_score(self._init_score_from_predictor(predictor, self.reference.data, self.used_indices))
        else:
            raise LightGBMError("Cannot set predictor after freed raw data, "
                                "set free_raw_data=False when construct Dataset to avoid this.")
        return self

    def get_ref_chain(self, ref_limit: int = 100) -> set:
        """This Dataset, its reference, the reference's reference, ... (stops at ref_limit or a loop)."""
        head, chain = self, set()
        while len(chain) < ref_limit and isinstance(head, Dataset):
            chain.add(head)
            if head.reference is None or head.reference in chain:
                break
            head = head.reference
        return chain

    def set_categorical_feature(self, categorical_feature: Any) -> "Dataset":
        if self.categorical_feature == categorical_feature:
            return self
        if self.handle is not None:
            raise LightGBMError("Cannot set categorical feature after constructed")
        self.categorical_feature = categorical_feature
        return self

    def set_feature_name(self, feature_name: Any) -> "Dataset":
        if feature_name != "auto":
            self.feature_name = feature_name
        if self.handle is not None and feature_name is not None and feature_name != "auto":
            names = [str(n) for n in feature_name]
            if len(names) != self.num_feature():
                raise ValueError(f"Length of feature_name({len(names)}) and num_feature({self.num_feature()}) don't match")
            arr = (ctypes.c_char_p * len(names))(*[n.encode("utf-8") for n in names])
            _check(_LIB.LGBM_DatasetSetFeatureNames(self.handle, arr, ctypes.c_int(len(names))))
        return self

    def get_feature_name(self) -> List[str]:
        if self.handle is None:
            raise LightGBMError("Cannot get feature_name before construct dataset")
        n = self.num_feature()
        return _get_names(lambda l, ol, bl, obl, arr: _LIB.LGBM_DatasetGetFeatureNames(self.handle, l, ol, bl, obl, arr), n)

    def num_data(self) -> int:
        if self.handle is None:
            raise LightGBMError("Cannot get num_data before construct dataset")
        out = ctypes.c_int(0)
        _check(_LIB.LGBM_DatasetGetNumData(self.handle, ctypes.byref(out)))
        return out.value

    def num_feature(self) -> int:
        if self.handle is None:
            raise LightGBMError("Cannot get num_feature before construct dataset")
        out = ctypes.c_int(0)
        _check(_LIB.LGBM_DatasetGetNumFeature(self.handle, ctypes.byref(out)))
        return out.value

    def feature_num_bin(self, feature: Union[int, str]) -> int:
        if isinstance(feature, str):
            feature = self.get_feature_name().index(feature)
        out = ctypes.c_int(0)
        _check(_LIB.LGBM_DatasetGetFeatureNumBin(self.handle, ctypes.c_int(feature), ctypes.byref(out)))
        return out.value

    def save_binary(self, filename: Union[str, Path]) -> "Dataset":
        self.construct()
        _check(_LIB.LGBM_DatasetSaveBinary(self.handle, _c_str(str(filename))))
        return self

    def _dump_text(self, filename: Union[str, Path]) -> "Dataset":
        self.construct()
        _check(_LIB.LGBM_DatasetDumpText(self.handle, _c_str(str(filename))))
        return self

    def add_features_from(self, other: "Dataset") -> "Dataset":
        """Append other's feature columns (both constructed; reference basic.py
        add_features_from). Raw data is merged where the two types allow it, else freed."""
        if self.handle is None or other.handle is None:
            raise ValueError("Both source and target Datasets must be constructed before adding features")
        _check(_LIB.LGBM_DatasetAddFeaturesFrom(self.handle, other.handle))
        was_none = self.data is None
        old_type = type(self.data).__name__
        od = other.data
        if od is None or _is_path(od):
            self.data = None
        elif self.data is not None:
            import scipy.sparse as _sp

            sd = self.data
            if isinstance(sd, np.ndarray):
                if isinstance(od, np.ndarray):
                    self.data = np.hstack((sd, od))
                elif _sp.issparse(od):
                    self.data = np.hstack((sd, od.toarray()))
                elif _is_pandas(od):
                    self.data = np.hstack((sd, od.values))
                else:
                    self.data = None
            elif _sp.issparse(sd):
                fmt = sd.getformat()
                if isinstance(od, np.ndarray) or _sp.issparse(od):
                    self.data = _sp.hstack((sd, od), format=fmt)
                elif _is_pandas(od):
                    self.data = _sp.hstack((sd, od.values), format=fmt)
                else:
                    self.data = None
            elif _is_pandas(sd):
                if isinstance(od, np.ndarray):
                    self.data = pd.concat((sd, pd.DataFrame(od)), axis=1, ignore_index=True)
                elif _sp.issparse(od):
                    self.data = pd.concat((sd, pd.DataFrame(od.toarray())), axis=1, ignore_index=True)
                elif _is_pandas(od):
                    self.data = pd.concat((sd, od), axis=1, ignore_index=True)
                else:
                    self.data = None
            else:
                self.data = None
        if self.data is None:
            msg = (f"Cannot add features from {type(od).__name__} type of raw data to {old_type} type of raw data.\n")
            msg += "Set free_raw_data=False when construct Dataset to avoid this" if was_none else "Freeing raw data"
            _log_warning(msg)
        self.feature_name = self.get_feature_name()
        _log_warning("Reseting categorical features.\n"
                     "You can set new categorical features via ``set_categorical_feature`` method")
        self.categorical_feature = "auto"
        self.pandas_categorical = None
        return self

    def _update_params(self, params: Optional[Dict[str, Any]]) -> "Dataset":
        """Merge ``params`` before construction. Once constructed, the Dataset keeps the
        parameters it was built with: new ones are only checked for changes to binning
        parameters, which rebuild the Dataset when its raw data is still held, else raise
        (reference basic.py Dataset._update_params)."""
        if not params:
            return self
        params = deepcopy(params)
        if self.handle is None:
            self._params_back_up = deepcopy(self.params)
            self.params.update(params)
            return self
        ret = _LIB.LGBM_DatasetUpdateParamChecking(_c_str(param_dict_to_str(self.params)),
                                                   _c_str(param_dict_to_str(params)))
        if ret != 0:
            if self.data is not None:
                self._params_back_up = deepcopy(self.params)
                self.params.update(params)
                self._free_handle()
            else:
                raise LightGBMError(_LIB.LGBM_GetLastError().decode("utf-8"))
        return self


def _get_names(fn: Callable, n: int) -> List[str]:
    buf_len = 256
    for _ in range(2):
        bufs = [ctypes.create_string_buffer(buf_len) for _ in range(max(n, 1))]
        ptrs = (ctypes.c_char_p * len(bufs))(*map(ctypes.addressof, bufs))
        out_len = ctypes.c_int(0)
        req = ctypes.c_size_t(0)
        _check(fn(ctypes.c_int(len(bufs)), ctypes.byref(out_len), ctypes.c_size_t(buf_len), ctypes.byref(req), ptrs))
        if req.value <= buf_len:
            return [bufs[i].value.decode("utf-8") for i in range(out_len.value)]
        buf_len = req.value
    return [bufs[i].value.decode("utf-8") for i in range(out_len.value)]


# reference basic.py:5268-5270 ("map@", not "map": "mape" is a loss); precision@k is a gain too
_HIGHER_BETTER_PREFIX = ("auc", "ndcg@", "map@", "average_precision", "precision@")


def _is_higher_better(name: str) -> bool:
    return name.startswith(_HIGHER_BETTER_PREFIX)


class Booster:
    """A gradient boosting model (training state + trees).

    Reference: python-package/lightgbm/basic.py Booster.
    """

    def __init__(self, params: Optional[Dict[str, Any]] = None, train_set: Optional[Dataset] = None,
                 model_file: Optional[Union[str, Path]] = None, model_str: Optional[str] = None):
        self.handle = ctypes.c_void_p()
        self.params = deepcopy(params) if params else {}
        self.best_iteration = 0
        self.best_score: Dict[str, Dict[str, float]] = {}
        self.name_valid_sets: List[str] = []
        self.valid_sets: List[Dataset] = []
        self._train_data_name = "training"
        self.train_set: Optional[Dataset] = None
        self.pandas_categorical = None
        self._num_class = 1
        self._eval_names: Optional[List[str]] = None
        self.__inner_predict_buffer: Dict[int, np.ndarray] = {}
        self._network = False
        if train_set is not None:
            if not isinstance(train_set, Dataset):
                raise TypeError(f"Training data should be Dataset instance, met {type(train_set).__name__}")
            # the socket mesh must exist before binning: distributed bin finding syncs the mappers
            self._setup_network()
            train_set._update_params(self.params)
            train_set.construct()
            self.train_set = train_set
            self.params.update(train_set.get_params())
            _check(_LIB.LGBM_BoosterCreate(train_set.handle, _c_str(param_dict_to_str(self.params)),
                                           ctypes.byref(self.handle)))
            if train_set._predictor is not None:
                # continued training: the init model's trees go first, its scores are the init score
                self._init_predictor = train_set._predictor
                _check(_LIB.LGBM_BoosterMerge(self.handle, self._init_predictor.handle))
            self.pandas_categorical = train_set.pandas_categorical
            self._num_class = self._get_num_class()
        elif model_file is not None:
            n_iter = ctypes.c_int(0)
            _check(_LIB.LGBM_BoosterCreateFromModelfile(_c_str(str(model_file)), ctypes.byref(n_iter),
                                                        ctypes.byref(self.handle)))
            self._num_class = self._get_num_class()
            self.pandas_categorical = _load_pandas_categorical(Path(model_file).read_text())
            self._params_from_model(params, "file")
        elif model_str is not None:
            self.model_from_string(model_str)
            self._params_from_model(params, "string")
        else:
            raise TypeError("Need at least one training dataset or model file or model string to create Booster instance")

    def _params_from_model(self, params: Optional[Dict[str, Any]], source: str) -> None:
        """Booster.params of a loaded model are the model's own parameters section (reference
        basic.py Booster.__init__ / _get_loaded_param); constructor params are ignored."""
        if params:
            _log_warning(f"Ignoring params argument, using parameters from model {source}.")
        s = _get_string(lambda n, ol, buf: _LIB.LGBM_BoosterGetLoadedParam(self.handle, ctypes.c_int64(n), ol, buf),
                        size=1 << 16)
        self.params = json.loads(s)

    def __del__(self):
        try:
            if self.handle is not None and self.handle.value:
                _LIB.LGBM_BoosterFree(self.handle)
                self.handle = None
            if getattr(self, "_network", False):
                _LIB.LGBM_NetworkFree()
                self._network = False
        except Exception:
            pass

    def _setup_network(self) -> None:
        """Socket mesh from `machines` / `num_machines` params (reference basic.py Booster.set_network)."""
        p = self.params
        machines = p.get("machines", p.get("workers", p.get("nodes")))
        num = int(p.get("num_machines", p.get("num_machine", 1)))
        if not machines or num <= 1:
            return
        if isinstance(machines, (list, tuple, set)):
            machines = ",".join(machines)
        port = int(p.get("local_listen_port", p.get("local_port", p.get("port", 12400))))
        timeout = int(p.get("time_out", 120))
        _check(_LIB.LGBM_NetworkInit(_c_str(str(machines)), ctypes.c_int(port), ctypes.c_int(timeout),
                                     ctypes.c_int(num)))
        self._network = True

    def set_network(self, machines: Union[List[str], set, str], local_listen_port: int = 12400,
                    listen_time_out: int = 120, num_machines: int = 1) -> "Booster":
        """Join the TCP socket mesh of the host parallel learners (reference Booster.set_network)."""
        if isinstance(machines, (list, set)):
            machines = ",".join(machines)
        _check(_LIB.LGBM_NetworkInit(_c_str(machines), ctypes.c_int(local_listen_port),
                                     ctypes.c_int(listen_time_out), ctypes.c_int(num_machines)))
        self._network = True
        return self

    def free_network(self) -> "Booster":
        if self._network:
            _check(_LIB.LGBM_NetworkFree())
            self._network = False
        return self

    def __copy__(self):
        return self.__deepcopy__(None)

    def __deepcopy__(self, memo):
        return Booster(model_str=self.model_to_string(num_iteration=-1))

    def __getstate__(self):
        state = self.__dict__.copy()
        state["handle"] = None
        state["_model_str"] = self.model_to_string(num_iteration=-1)
        state["train_set"] = None
        state["valid_sets"] = []
        return state

    def __setstate__(self, state):
        ms = state.pop("_model_str")
        self.__dict__.update(state)
        self.handle = ctypes.c_void_p()
        n_iter = ctypes.c_int(0)
        _check(_LIB.LGBM_BoosterLoadModelFromString(_c_str(ms), ctypes.byref(n_iter), ctypes.byref(self.handle)))

    def _get_num_class(self) -> int:
        out = ctypes.c_int(0)
        _check(_LIB.LGBM_BoosterGetNumClasses(self.handle, ctypes.byref(out)))
        return out.value

    # ------------------------------------------------------------------ training
    def free_dataset(self) -> "Booster":
        self.train_set = None
        self.valid_sets = []
        return self

    def set_train_data_name(self, name: str) -> "Booster":
        self._train_data_name = name
        return self

    def add_valid(self, data: Dataset, name: str) -> "Booster":
        if data.reference is not self.train_set and self.train_set is not None and data is not self.train_set:
            if data.reference is None:
                data.set_reference(self.train_set)
        if data.handle is None:
            data.params = {**self.params, **data.params}
        data.construct()
        _check(_LIB.LGBM_BoosterAddValidData(self.handle, data.handle))
        self.valid_sets.append(data)
        self.name_valid_sets.append(name)
        return self

    def reset_parameter(self, params: Dict[str, Any]) -> "Booster":
        s = param_dict_to_str(params)
        if s:
            _check(_LIB.LGBM_BoosterResetParameter(self.handle, _c_str(s)))
        self.params.update(params)
        return self

    def update(self, train_set: Optional[Dataset] = None, fobj: Optional[Callable] = None) -> bool:
        if train_set is not None and train_set is not self.train_set:
            train_set.construct()
            _check(_LIB.LGBM_BoosterResetTrainingData(self.handle, train_set.handle))
            self.train_set = train_set
            self.__inner_predict_buffer.clear()
        finished = ctypes.c_int(0)
        if fobj is None:
            _check(_LIB.LGBM_BoosterUpdateOneIter(self.handle, ctypes.byref(finished)))
        else:
            grad, hess = fobj(self.__inner_predict(0), self.train_set)
            return self.__boost(grad, hess)
        self.__inner_predict_buffer.clear()
        return finished.value == 1

    def __boost(self, grad: Any, hess: Any) -> bool:
        g = np.ascontiguousarray(np.asarray(grad, dtype=np.float32).T.ravel() if np.ndim(grad) == 2 else grad,
                                 dtype=np.float32)
        h = np.ascontiguousarray(np.asarray(hess, dtype=np.float32).T.ravel() if np.ndim(hess) == 2 else hess,
                                 dtype=np.float32)
        if g.size != h.size:
            raise ValueError(f"Lengths of gradient ({g.size}) and Hessian ({h.size}) don't match")
        finished = ctypes.c_int(0)
        _check(_LIB.LGBM_BoosterUpdateOneIterCustom(self.handle, g.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                                    h.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                                    ctypes.byref(finished)))
        self.__inner_predict_buffer.clear()
        return finished.value == 1

    def rollback_one_iter(self) -> "Booster":
        _check(_LIB.LGBM_BoosterRollbackOneIter(self.handle))
        self.__inner_predict_buffer.clear()
        return self

    def current_iteration(self) -> int:
        out = ctypes.c_int(0)
        _check(_LIB.LGBM_BoosterGetCurrentIteration(self.handle, ctypes.byref(out)))
        return out.value

    def num_model_per_iteration(self) -> int:
        out = ctypes.c_int(0)
        _check(_LIB.LGBM_BoosterNumModelPerIteration(self.handle, ctypes.byref(out)))
        return out.value

    def num_trees(self) -> int:
        out = ctypes.c_int(0)
        _check(_LIB.LGBM_BoosterNumberOfTotalModel(self.handle, ctypes.byref(out)))
        return out.value

    def upper_bound(self) -> float:
        out = ctypes.c_double(0)
        _check(_LIB.LGBM_BoosterGetUpperBoundValue(self.handle, ctypes.byref(out)))
        return out.value

    def lower_bound(self) -> float:
        out = ctypes.c_double(0)
        _check(_LIB.LGBM_BoosterGetLowerBoundValue(self.handle, ctypes.byref(out)))
        return out.value

    def device_name(self) -> str:
        return _get_string(lambda n, ol, buf: _LIB.LGBM_BoosterGetDeviceName(self.handle, ctypes.c_int64(n), ol, buf))

    # ------------------------------------------------------------------ evaluation
    def __inner_predict(self, data_idx: int) -> np.ndarray:
        if data_idx not in self.__inner_predict_buffer:
            n = ctypes.c_int64(0)
            _check(_LIB.LGBM_BoosterGetNumPredict(self.handle, ctypes.c_int(data_idx), ctypes.byref(n)))
            out = np.empty(n.value, dtype=np.float64)
            out_len = ctypes.c_int64(0)
            _check(_LIB.LGBM_BoosterGetPredict(self.handle, ctypes.c_int(data_idx), ctypes.byref(out_len),
                                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
            k = self._num_class
            if k > 1:
                out = out.reshape(k, -1).T
            self.__inner_predict_buffer[data_idx] = out
        return self.__inner_predict_buffer[data_idx]

    def _eval_names_list(self) -> List[str]:
        if self._eval_names is None:
            cnt = ctypes.c_int(0)
            _check(_LIB.LGBM_BoosterGetEvalCounts(self.handle, ctypes.byref(cnt)))
            self._eval_names = _get_names(
                lambda l, ol, bl, obl, arr: _LIB.LGBM_BoosterGetEvalNames(self.handle, l, ol, bl, obl, arr), cnt.value)
        return self._eval_names

    def __inner_eval(self, data_name: str, data_idx: int, feval: Any = None) -> List[Tuple[str, str, float, bool]]:
        ret = []
        names = self._eval_names_list()
        if names:
            res = np.zeros(len(names), dtype=np.float64)
            out_len = ctypes.c_int(0)
            _check(_LIB.LGBM_BoosterGetEval(self.handle, ctypes.c_int(data_idx), ctypes.byref(out_len),
                                            res.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
            for i in range(out_len.value):
                ret.append((data_name, names[i], float(res[i]), _is_higher_better(names[i])))
        if feval is not None:
            data = self.train_set if data_idx == 0 else self.valid_sets[data_idx - 1]
            fevals = feval if isinstance(feval, (list, tuple)) else [feval]
            preds = self.__inner_predict(data_idx)
            for fe in fevals:
                out = fe(preds, data)
                outs = out if isinstance(out, list) else [out]
                for name, val, hib in outs:
                    ret.append((data_name, name, float(val), bool(hib)))
        return ret

    def eval(self, data: Dataset, name: str, feval: Any = None) -> List[Tuple[str, str, float, bool]]:
        if data is self.train_set:
            return self.__inner_eval(self._train_data_name, 0, feval)
        for i, v in enumerate(self.valid_sets):
            if data is v:
                return self.__inner_eval(name, i + 1, feval)
        self.add_valid(data, name)
        return self.__inner_eval(name, len(self.valid_sets), feval)

    def eval_train(self, feval: Any = None) -> List[Tuple[str, str, float, bool]]:
        return self.__inner_eval(self._train_data_name, 0, feval)

    def eval_valid(self, feval: Any = None) -> List[Tuple[str, str, float, bool]]:
        out = []
        for i, name in enumerate(self.name_valid_sets):
            out.extend(self.__inner_eval(name, i + 1, feval))
        return out

    # ------------------------------------------------------------------ prediction
    def predict(self, data: Any, start_iteration: int = 0, num_iteration: Optional[int] = None,
                raw_score: bool = False, pred_leaf: bool = False, pred_contrib: bool = False,
                data_has_header: bool = False, validate_features: bool = False, **kwargs: Any) -> np.ndarray:
        if isinstance(data, Dataset):
            raise TypeError("Cannot use Dataset instance for prediction, please use raw data instead")
        if num_iteration is None:
            num_iteration = self.best_iteration if self.best_iteration > 0 else -1
        ptype = C_API_PREDICT_NORMAL
        if raw_score:
            ptype = C_API_PREDICT_RAW_SCORE
        if pred_leaf:
            ptype = C_API_PREDICT_LEAF_INDEX
        if pred_contrib:
            ptype = C_API_PREDICT_CONTRIB
        params = _c_str(param_dict_to_str(kwargs))
        if _is_path(data):
            import tempfile

            with tempfile.NamedTemporaryFile(suffix=".txt", delete=False) as f:
                tmp = f.name
            try:
                _check(_LIB.LGBM_BoosterPredictForFile(self.handle, _c_str(str(data)), ctypes.c_int(int(data_has_header)),
                                                       ctypes.c_int(ptype), ctypes.c_int(start_iteration),
                                                       ctypes.c_int(num_iteration), params, _c_str(tmp)))
                res = np.loadtxt(tmp, dtype=np.float64, ndmin=2)
            finally:
                os.unlink(tmp)
            return res[:, 0] if res.shape[1] == 1 else res
        if _is_pandas(data):
            if validate_features:
                names = [str(c) for c in data.columns]
                arr = (ctypes.c_char_p * len(names))(*[n.encode("utf-8") for n in names])
                _check(_LIB.LGBM_BoosterValidateFeatureNames(self.handle, arr, ctypes.c_int(len(names))))
            data = _pandas_to_numpy(data, "auto", self.pandas_categorical)[0]
        if _is_arrow(data):
            nrow = data.num_rows
            n_pred = ctypes.c_int64(0)
            _check(_LIB.LGBM_BoosterCalcNumPredict(self.handle, ctypes.c_int(nrow), ctypes.c_int(ptype),
                                                   ctypes.c_int(start_iteration), ctypes.c_int(num_iteration),
                                                   ctypes.byref(n_pred)))
            out = np.empty(n_pred.value, dtype=np.float64)
            out_len = ctypes.c_int64(0)
            with _ArrowExport(data) as ex:
                _check(_LIB.LGBM_BoosterPredictForArrow(self.handle, ctypes.c_int64(ex.n), ex.chunks,
                                                        ctypes.byref(ex.schema), ctypes.c_int(ptype),
                                                        ctypes.c_int(start_iteration), ctypes.c_int(num_iteration),
                                                        params, ctypes.byref(out_len),
                                                        out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
            return self._shape_pred(out, nrow, ptype)
        if _is_sparse(data) and pred_contrib:
            return self._predict_sparse_contrib(data, start_iteration, num_iteration, params)
        if _is_sparse(data):
            return self._predict_sparse(data, ptype, start_iteration, num_iteration, params)
        mat, dtype = _to_float_matrix(data if not isinstance(data, list) else np.asarray(data))
        nrow = mat.shape[0]
        n_pred = ctypes.c_int64(0)
        _check(_LIB.LGBM_BoosterCalcNumPredict(self.handle, ctypes.c_int(nrow), ctypes.c_int(ptype),
                                               ctypes.c_int(start_iteration), ctypes.c_int(num_iteration),
                                               ctypes.byref(n_pred)))
        out = np.empty(n_pred.value, dtype=np.float64)
        out_len = ctypes.c_int64(0)
        _check(_LIB.LGBM_BoosterPredictForMat(self.handle, mat.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(dtype),
                                              ctypes.c_int32(nrow), ctypes.c_int32(mat.shape[1]), ctypes.c_int(1),
                                              ctypes.c_int(ptype), ctypes.c_int(start_iteration),
                                              ctypes.c_int(num_iteration), params, ctypes.byref(out_len),
                                              out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        return self._shape_pred(out, nrow, ptype)

    def _predict_sparse(self, data, ptype, start_iteration, num_iteration, params) -> np.ndarray:
        csr = data.tocsr()
        nrow = csr.shape[0]
        n_pred = ctypes.c_int64(0)
        _check(_LIB.LGBM_BoosterCalcNumPredict(self.handle, ctypes.c_int(nrow), ctypes.c_int(ptype),
                                               ctypes.c_int(start_iteration), ctypes.c_int(num_iteration),
                                               ctypes.byref(n_pred)))
        out = np.empty(n_pred.value, dtype=np.float64)
        out_len = ctypes.c_int64(0)
        indptr, ip_type = Dataset._indptr(csr.indptr)
        vals, vtype = Dataset._values(csr.data)
        indices = np.ascontiguousarray(csr.indices, dtype=np.int32)
        _check(_LIB.LGBM_BoosterPredictForCSR(self.handle, indptr.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(ip_type),
                                              indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                              vals.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(vtype),
                                              ctypes.c_int64(indptr.size), ctypes.c_int64(vals.size),
                                              ctypes.c_int64(csr.shape[1]), ctypes.c_int(ptype),
                                              ctypes.c_int(start_iteration), ctypes.c_int(num_iteration), params,
                                              ctypes.byref(out_len), out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        return self._shape_pred(out, nrow, ptype)

    def _predict_sparse_contrib(self, data, start_iteration, num_iteration, params):
        """SHAP values of sparse input as sparse matrices (one per class when multiclass),
        in the input's format (reference basic.py __inner_predict_sparse_csr/csc)."""
        is_csc = data.format == "csc"
        mat = data if data.format in ("csr", "csc") else data.tocsr()
        indptr, ip_type = Dataset._indptr(mat.indptr)
        vals, vtype = Dataset._values(mat.data)
        indices = np.ascontiguousarray(mat.indices, dtype=np.int32)
        out_len = (ctypes.c_int64 * 2)()
        out_ptr, out_idx, out_data = ctypes.c_void_p(), ctypes.POINTER(ctypes.c_int32)(), ctypes.c_void_p()
        other = mat.shape[0] if is_csc else mat.shape[1]
        _check(_LIB.LGBM_BoosterPredictSparseOutput(
            self.handle, indptr.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(ip_type),
            indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), vals.ctypes.data_as(ctypes.c_void_p),
            ctypes.c_int(vtype), ctypes.c_int64(indptr.size), ctypes.c_int64(vals.size), ctypes.c_int64(other),
            ctypes.c_int(C_API_PREDICT_CONTRIB), ctypes.c_int(start_iteration), ctypes.c_int(num_iteration), params,
            ctypes.c_int(1 if is_csc else 0), out_len, ctypes.byref(out_ptr), ctypes.byref(out_idx),
            ctypes.byref(out_data)))
        try:
            nnz, nptr = out_len[0], out_len[1]
            pt = ctypes.c_int32 if ip_type == C_API_DTYPE_INT32 else ctypes.c_int64
            dt = ctypes.c_float if vtype == C_API_DTYPE_FLOAT32 else ctypes.c_double
            ptr = np.ctypeslib.as_array(ctypes.cast(out_ptr, ctypes.POINTER(pt)), shape=(nptr,)).copy()
            idx = np.ctypeslib.as_array(out_idx, shape=(max(nnz, 1),))[:nnz].copy()
            val = np.ctypeslib.as_array(ctypes.cast(out_data, ctypes.POINTER(dt)), shape=(max(nnz, 1),))[:nnz].copy()
        finally:
            _check(_LIB.LGBM_BoosterFreePredictSparse(out_ptr, out_idx, out_data, ctypes.c_int(ip_type),
                                                      ctypes.c_int(vtype)))
        k = self.num_model_per_iteration()
        nrow = mat.shape[0]
        width = self.num_feature() + 1
        outer = width if is_csc else nrow
        shape = (nrow, width)
        mats, off = [], 0
        for c in range(k):
            p = ptr[c * (outer + 1):(c + 1) * (outer + 1)]
            n = int(p[-1])
            seg_i, seg_v = idx[off:off + n], val[off:off + n]
            off += n
            mats.append(sp.csc_matrix((seg_v, seg_i, p), shape=shape) if is_csc else
                        sp.csr_matrix((seg_v, seg_i, p), shape=shape))
        return mats[0] if k == 1 else mats

    def _shape_pred(self, out: np.ndarray, nrow: int, ptype: int) -> np.ndarray:
        if nrow == 0:
            return out
        per = out.size // nrow
        # leaf indices and contributions are always (nrow, k) (reference _InnerPredictor)
        if per == 1 and ptype not in (C_API_PREDICT_LEAF_INDEX, C_API_PREDICT_CONTRIB):
            return out
        res = out.reshape(nrow, per)
        if ptype == C_API_PREDICT_LEAF_INDEX:
            return res.astype(np.int32)
        return res

    # ------------------------------------------------------------------ model IO
    def save_model(self, filename: Union[str, Path], num_iteration: Optional[int] = None, start_iteration: int = 0,
                   importance_type: str = "split") -> "Booster":
        if num_iteration is None:
            num_iteration = self.best_iteration
        it = C_API_FEATURE_IMPORTANCE_GAIN if importance_type == "gain" else C_API_FEATURE_IMPORTANCE_SPLIT
        _check(_LIB.LGBM_BoosterSaveModel(self.handle, ctypes.c_int(start_iteration), ctypes.c_int(num_iteration),
                                          ctypes.c_int(it), _c_str(str(filename))))
        if self.pandas_categorical:
            with open(filename, "a") as f:
                f.write(_dump_pandas_categorical(self.pandas_categorical))
        return self

    def model_to_string(self, num_iteration: Optional[int] = None, start_iteration: int = 0,
                        importance_type: str = "split") -> str:
        if num_iteration is None:
            num_iteration = self.best_iteration
        it = C_API_FEATURE_IMPORTANCE_GAIN if importance_type == "gain" else C_API_FEATURE_IMPORTANCE_SPLIT
        s = _get_string(lambda n, ol, buf: _LIB.LGBM_BoosterSaveModelToString(
            self.handle, ctypes.c_int(start_iteration), ctypes.c_int(num_iteration), ctypes.c_int(it),
            ctypes.c_int64(n), ol, buf), size=1 << 20)
        if self.pandas_categorical:
            s += _dump_pandas_categorical(self.pandas_categorical)
        return s

    def model_from_string(self, model_str: str) -> "Booster":
        if self.handle is not None and self.handle.value:
            _check(_LIB.LGBM_BoosterFree(self.handle))
        self.handle = ctypes.c_void_p()
        n_iter = ctypes.c_int(0)
        _check(_LIB.LGBM_BoosterLoadModelFromString(_c_str(model_str), ctypes.byref(n_iter), ctypes.byref(self.handle)))
        self._num_class = self._get_num_class()
        self.pandas_categorical = _load_pandas_categorical(model_str)
        return self

    def dump_model(self, num_iteration: Optional[int] = None, start_iteration: int = 0,
                   importance_type: str = "split", object_hook: Optional[Callable] = None) -> Dict[str, Any]:
        if num_iteration is None:
            num_iteration = self.best_iteration
        it = C_API_FEATURE_IMPORTANCE_GAIN if importance_type == "gain" else C_API_FEATURE_IMPORTANCE_SPLIT
        s = _get_string(lambda n, ol, buf: _LIB.LGBM_BoosterDumpModel(
            self.handle, ctypes.c_int(start_iteration), ctypes.c_int(num_iteration), ctypes.c_int(it),
            ctypes.c_int64(n), ol, buf), size=1 << 20)
        ret = json.loads(s, object_hook=object_hook)
        ret["pandas_categorical"] = self.pandas_categorical
        return ret

    def model_to_if_else(self, num_iteration: int = -1) -> str:
        return _get_string(lambda n, ol, buf: _LIB.LGBM_BoosterConvertModelToIfElse(
            self.handle, ctypes.c_int(num_iteration), ctypes.c_int64(n), ol, buf), size=1 << 20)

    def shuffle_models(self, start_iteration: int = 0, end_iteration: int = -1) -> "Booster":
        _check(_LIB.LGBM_BoosterShuffleModels(self.handle, ctypes.c_int(start_iteration), ctypes.c_int(end_iteration)))
        return self

    def merge(self, other: "Booster") -> "Booster":
        _check(_LIB.LGBM_BoosterMerge(self.handle, other.handle))
        return self

    def refit(self, data: Any, label: Any, decay_rate: float = 0.9, reference: Optional[Dataset] = None,
              weight: Any = None, group: Any = None, init_score: Any = None, dataset_params: Optional[Dict] = None,
              free_raw_data: bool = True, validate_features: bool = False, **kwargs: Any) -> "Booster":
        leaf_preds = self.predict(data, start_iteration=0, num_iteration=-1, pred_leaf=True,
                                  validate_features=validate_features)
        nrow = leaf_preds.shape[0]
        leaf_preds = np.ascontiguousarray(leaf_preds.reshape(nrow, -1), dtype=np.int32)
        params = dict(self.params)
        params["refit_decay_rate"] = decay_rate
        params.update(kwargs)
        train = Dataset(data, label=label, weight=weight, group=group, init_score=init_score,
                        params=dataset_params or {}, free_raw_data=free_raw_data,
                        categorical_feature=self.params.get("categorical_feature", "auto"))
        new = Booster(params=params, train_set=train)
        _check(_LIB.LGBM_BoosterMerge(new.handle, self.handle))
        _check(_LIB.LGBM_BoosterRefit(new.handle, leaf_preds.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                      ctypes.c_int32(nrow), ctypes.c_int32(leaf_preds.shape[1])))
        new.pandas_categorical = self.pandas_categorical
        return new

    # ------------------------------------------------------------------ introspection
    def num_feature(self) -> int:
        out = ctypes.c_int(0)
        _check(_LIB.LGBM_BoosterGetNumFeature(self.handle, ctypes.byref(out)))
        return out.value

    def feature_name(self) -> List[str]:
        n = self.num_feature()
        return _get_names(lambda l, ol, bl, obl, arr: _LIB.LGBM_BoosterGetFeatureNames(self.handle, l, ol, bl, obl, arr),
                          n)

    def feature_importance(self, importance_type: str = "split", iteration: Optional[int] = None) -> np.ndarray:
        if iteration is None:
            iteration = self.best_iteration
        it = C_API_FEATURE_IMPORTANCE_GAIN if importance_type == "gain" else C_API_FEATURE_IMPORTANCE_SPLIT
        out = np.zeros(self.num_feature(), dtype=np.float64)
        _check(_LIB.LGBM_BoosterFeatureImportance(self.handle, ctypes.c_int(iteration), ctypes.c_int(it),
                                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        return out.astype(np.int32) if importance_type == "split" else out

    def get_leaf_output(self, tree_id: int, leaf_id: int) -> float:
        out = ctypes.c_double(0)
        _check(_LIB.LGBM_BoosterGetLeafValue(self.handle, ctypes.c_int(tree_id), ctypes.c_int(leaf_id),
                                             ctypes.byref(out)))
        return out.value

    def set_leaf_output(self, tree_id: int, leaf_id: int, value: float) -> "Booster":
        _check(_LIB.LGBM_BoosterSetLeafValue(self.handle, ctypes.c_int(tree_id), ctypes.c_int(leaf_id),
                                             ctypes.c_double(value)))
        return self

    def get_split_value_histogram(self, feature: Union[int, str], bins: Any = None, xgboost_style: bool = False):
        model = self.dump_model()
        names = model["feature_names"]
        fidx = names.index(feature) if isinstance(feature, str) else int(feature)
        values: List[float] = []

        def walk(node):
            if "split_index" in node:
                if node["split_feature"] == fidx:
                    if isinstance(node["threshold"], str):
                        raise LightGBMError("Cannot compute split value histogram for the categorical feature")
                    values.append(node["threshold"])
                walk(node["left_child"])
                walk(node["right_child"])

        for t in model["tree_info"]:
            walk(t["tree_structure"])
        if bins is None or (isinstance(bins, int) and xgboost_style):
            n_unique = len(np.unique(values))
            bins = max(min(n_unique, bins) if bins is not None else n_unique, 1)
        hist, edges = np.histogram(values, bins=bins)
        if xgboost_style:
            ret = np.column_stack((edges[1:], hist))
            ret = ret[ret[:, 1] > 0]
            if pd is not None:
                return pd.DataFrame(ret, columns=["SplitValue", "Count"])
            return ret
        return hist, edges

    def trees_to_dataframe(self):
        if pd is None:
            raise LightGBMError("This method cannot be run without pandas installed.")
        model = self.dump_model()
        names = model["feature_names"]
        rows = []

        def walk(node, tree_index, depth, parent):
            is_split = "split_index" in node
            nid = (f"{tree_index}-S{node['split_index']}" if is_split else f"{tree_index}-L{node.get('leaf_index', 0)}")
            row = {"tree_index": tree_index, "node_depth": depth, "node_index": nid, "left_child": None,
                   "right_child": None, "parent_index": parent,
                   "split_feature": names[node["split_feature"]] if is_split else None,
                   "split_gain": node.get("split_gain") if is_split else None,
                   "threshold": node.get("threshold") if is_split else None,
                   "decision_type": node.get("decision_type") if is_split else None,
                   "missing_direction": ("left" if node.get("default_left") else "right") if is_split else None,
                   "missing_type": node.get("missing_type") if is_split else None,
                   "value": node["internal_value"] if is_split else node["leaf_value"],
                   "weight": node["internal_weight"] if is_split else node.get("leaf_weight"),
                   "count": node["internal_count"] if is_split else node.get("leaf_count")}
            if not is_split and "leaf_weight" not in node:
                # a single-leaf tree has no weight record; the reference leaves both unset
                # (basic.py trees_to_dataframe _is_single_node_tree)
                row["weight"] = row["count"] = None
            rows.append(row)
            if is_split:
                lrow = walk(node["left_child"], tree_index, depth + 1, nid)
                rrow = walk(node["right_child"], tree_index, depth + 1, nid)
                row["left_child"], row["right_child"] = lrow, rrow
            return nid

        for t in model["tree_info"]:
            walk(t["tree_structure"], t["tree_index"], 1, None)
        return pd.DataFrame(rows)


def _dump_pandas_categorical(pc) -> str:
    return "\npandas_categorical:" + json.dumps(pc, default=lambda o: o.item() if hasattr(o, "item") else str(o)) + "\n"


def _load_pandas_categorical(model_str: str):
    key = "pandas_categorical:"
    pos = model_str.rfind(key)
    if pos < 0:
        return None
    line = model_str[pos + len(key):].strip().splitlines()[0] if model_str[pos + len(key):].strip() else "null"
    try:
        return json.loads(line)
    except ValueError:
        return None
