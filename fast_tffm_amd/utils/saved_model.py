"""TensorFlow SavedModel export of the serving graph, written without TensorFlow.

Reference: ``run.py generate`` builds the serving graph of tffm/fm_model.py:195-265
(``serving_parser``: ``data_lines`` -> StringSplit(' ') -> StringSplit(':') ->
StringToNumber ids / values -> SparseToDense; ``serving_scorer``: embedding_lookup of the ids
in ``vocab_block_i`` with the "mod" partition strategy, then the dense FM score) and saves it
with ``SavedModelBuilder`` under tag ``serve``, signature ``serving_default`` (input
``data_lines``, output ``scores``, method ``tensorflow/serving/predict``; run_tffm.py:93-120).

This module emits the same graph -- standard TF1 ops only, node for node the structure the
reference's Python builds -- as a ``saved_model.pb`` (SavedModel / MetaGraphDef / GraphDef /
SaverDef / SignatureDef protobufs encoded by hand: no generated classes exist in this image)
and the variables as a V2 tensor bundle (``variables/variables.{index,data-00000-of-00001}``,
utils/tf_bundle.py) restored by the graph's ``save/restore_all`` op.

Parity status: unpinned against TensorFlow itself (not installable here).  ``run_graph``
below is an independent numpy interpreter of the emitted GraphDef (it decodes the protobuf
and evaluates every node by the TF op's documented semantics); tests/test_saved_model.py runs
exported models through it and compares the scores with the native predictor.
"""

from __future__ import annotations

import os
import struct

import numpy as np

from .tf_bundle import _field, _parse_pb, _pb_bytes, _pb_varint, _read_varint, _varint, read_bundle, write_bundle

# tensorflow/core/framework/types.proto
DT_FLOAT, DT_INT32, DT_STRING, DT_INT64, DT_BOOL = 1, 3, 7, 9, 10
_NP_OF = {DT_FLOAT: np.float32, DT_INT32: np.int32, DT_INT64: np.int64, DT_BOOL: np.bool_}
_DT_OF = {np.dtype(v): k for k, v in _NP_OF.items()}
GRAPH_PRODUCER = 134          # GraphDef version of TF 1.15 (the reference targets TF 1.x)
SIGNATURE_KEY = "serving_default"
PREDICT_METHOD = "tensorflow/serving/predict"
SERVE_TAG = "serve"


# --------------------------------------------------------------------------- protobuf encoding
def _field5(num: int) -> bytes:
    return _field(num, 5)


def _map_entry(num: int, key: str, value: bytes) -> bytes:
    return _pb_bytes(num, _pb_bytes(1, key.encode()) + _pb_bytes(2, value))


def shape_proto(dims: list[int] | None) -> bytes:
    """TensorShapeProto: dim = 2 {size = 1}, unknown_rank = 3."""
    if dims is None:
        return _pb_varint(3, 1)
    return b"".join(_pb_bytes(2, _pb_varint(1, d) if d >= 0 else _pb_varint(1, (1 << 64) + d)) for d in dims)


def tensor_proto(value) -> bytes:
    """TensorProto: dtype = 1, tensor_shape = 2, tensor_content = 4 (numeric), string_val = 8."""
    if isinstance(value, (bytes, str)) or (isinstance(value, (list, tuple)) and value
                                           and isinstance(value[0], (bytes, str))):
        vals = [value] if isinstance(value, (bytes, str)) else list(value)
        vals = [v.encode() if isinstance(v, str) else v for v in vals]
        shape = [] if isinstance(value, (bytes, str)) else [len(vals)]
        return (_pb_varint(1, DT_STRING) + _pb_bytes(2, shape_proto(shape))
                + b"".join(_pb_bytes(8, v) for v in vals))
    a = np.asarray(value)
    if a.dtype == np.float64:
        a = a.astype(np.float32)
    return (_pb_varint(1, _DT_OF[a.dtype]) + _pb_bytes(2, shape_proto(list(a.shape)))
            + _pb_bytes(4, a.astype(a.dtype.newbyteorder("<")).tobytes()))


def attr_proto(v) -> bytes:
    """AttrValue: list = 1, s = 2, i = 3, f = 4, b = 5, type = 6, shape = 7, tensor = 8."""
    kind, x = v
    if kind == "s":
        return _pb_bytes(2, x.encode() if isinstance(x, str) else x)
    if kind == "i":
        return _pb_varint(3, x & ((1 << 64) - 1))
    if kind == "f":
        return _field5(4) + struct.pack("<f", x)
    if kind == "b":
        return _pb_varint(5, int(bool(x)))
    if kind == "type":
        return _pb_varint(6, x)
    if kind == "shape":
        return _pb_bytes(7, shape_proto(x))
    if kind == "tensor":
        return _pb_bytes(8, tensor_proto(x))
    if kind == "types":  # ListValue.type = 6 (packed)
        return _pb_bytes(1, _pb_bytes(6, b"".join(_varint(t) for t in x)))
    raise ValueError(kind)


class GraphBuilder:
    """NodeDefs (name = 1, op = 2, input = 3, attr = 5) of one GraphDef."""

    def __init__(self):
        self.nodes: list[tuple[str, str, list[str], dict]] = []
        self.names: set[str] = set()

    def add(self, name: str, op: str, inputs: list[str] | None = None, **attrs) -> str:
        if name in self.names:
            raise ValueError(f"duplicate node {name}")
        self.names.add(name)
        self.nodes.append((name, op, list(inputs or []), attrs))
        return name

    def const(self, name: str, value, dtype: int | None = None) -> str:
        if isinstance(value, (bytes, str)) or (isinstance(value, list) and value
                                               and isinstance(value[0], (str, bytes))):
            dt = DT_STRING
        else:
            a = np.asarray(value, dtype=_NP_OF[dtype] if dtype else None)
            value, dt = a, _DT_OF[a.dtype if a.dtype != np.float64 else np.dtype(np.float32)]
        return self.add(name, "Const", dtype=("type", dt), value=("tensor", value))

    def graph_def(self) -> bytes:
        out = b""
        for name, op, inputs, attrs in self.nodes:
            nd = _pb_bytes(1, name.encode()) + _pb_bytes(2, op.encode())
            nd += b"".join(_pb_bytes(3, i.encode()) for i in inputs)
            nd += b"".join(_map_entry(5, k, attr_proto(v)) for k, v in sorted(attrs.items()))
            out += _pb_bytes(1, nd)
        return out + _pb_bytes(4, _pb_varint(1, GRAPH_PRODUCER))


# --------------------------------------------------------------------------- the serving graph
def build_serving_graph(vocabulary_size: int, block_num: int, factor_num: int,
                        global_bias: float | None = None) -> tuple[GraphBuilder, str, str]:
    """The reference's serving graph (fm_model.py:195-265); returns (graph, input, output) tensor names."""
    g = GraphBuilder()
    T = lambda t: ("type", t)  # noqa: E731
    rows = vocabulary_size // block_num + 1
    # serving_parser
    g.add("test_data", "Placeholder", dtype=T(DT_STRING), shape=("shape", None))
    g.const("Reshape/shape", [-1], DT_INT32)
    g.add("Reshape", "Reshape", ["test_data", "Reshape/shape"], T=T(DT_STRING), Tshape=T(DT_INT32))
    g.const("StringSplit/delimiter", " ")
    g.add("StringSplit", "StringSplit", ["Reshape", "StringSplit/delimiter"], skip_empty=("b", True))
    g.const("StringSplit_1/delimiter", ":")
    g.add("StringSplit_1", "StringSplit", ["StringSplit:1", "StringSplit_1/delimiter"], skip_empty=("b", True))
    g.const("Reshape_1/shape", [-1, 2], DT_INT32)
    g.add("Reshape_1", "Reshape", ["StringSplit_1:1", "Reshape_1/shape"], T=T(DT_STRING), Tshape=T(DT_INT32))
    for k, (col, out_t) in enumerate(((0, DT_INT64), (1, DT_FLOAT))):
        sfx = "" if k == 0 else "_1"
        g.const(f"Slice{sfx}/begin", [0, col], DT_INT32)
        g.const(f"Slice{sfx}/size", [-1, 1], DT_INT32)
        g.add(f"Slice{sfx}", "Slice", ["Reshape_1", f"Slice{sfx}/begin", f"Slice{sfx}/size"], T=T(DT_STRING),
              Index=T(DT_INT32))
        r = f"Reshape_{2 + k}"
        g.const(f"{r}/shape", [-1], DT_INT32)
        g.add(r, "Reshape", [f"Slice{sfx}", f"{r}/shape"], T=T(DT_STRING), Tshape=T(DT_INT32))
        g.add(f"StringToNumber{sfx}", "StringToNumber", [r], out_type=T(out_t))
        g.const(f"SparseToDense{sfx}/default_value", np.zeros((), _NP_OF[out_t]))
        g.add(f"SparseToDense{sfx}", "SparseToDense",
              ["StringSplit:0", "StringSplit:2", f"StringToNumber{sfx}", f"SparseToDense{sfx}/default_value"],
              T=T(out_t), Tindices=T(DT_INT64), validate_indices=("b", True))
    # serving_scorer: variables + embedding_lookup (partition_strategy "mod")
    for i in range(block_num):
        g.add(f"vocab_block_{i}", "VariableV2", shape=("shape", [rows, factor_num + 1]), dtype=T(DT_FLOAT),
              container=("s", ""), shared_name=("s", ""))
        g.add(f"vocab_block_{i}/read", "Identity", [f"vocab_block_{i}"], T=T(DT_FLOAT))
    g.const("Reshape_4/shape", [-1], DT_INT32)
    g.add("Reshape_4", "Reshape", ["SparseToDense", "Reshape_4/shape"], T=T(DT_INT64), Tshape=T(DT_INT32))
    el = "embedding_lookup"
    g.const(f"{el}/axis", 0, DT_INT32)
    if block_num == 1:
        g.add(el, "GatherV2", ["vocab_block_0/read", "Reshape_4", f"{el}/axis"], Tparams=T(DT_FLOAT),
              Tindices=T(DT_INT64), Taxis=T(DT_INT32), batch_dims=("i", 0))
        params = el
    else:
        g.const(f"{el}/mod/y", block_num, DT_INT64)
        g.add(f"{el}/mod", "FloorMod", ["Reshape_4", f"{el}/mod/y"], T=T(DT_INT64))
        g.add(f"{el}/Cast", "Cast", [f"{el}/mod"], SrcT=T(DT_INT64), DstT=T(DT_INT32), Truncate=("b", False))
        g.const(f"{el}/floordiv/y", block_num, DT_INT64)
        g.add(f"{el}/floordiv", "FloorDiv", ["Reshape_4", f"{el}/floordiv/y"], T=T(DT_INT64))
        g.add(f"{el}/DynamicPartition", "DynamicPartition", [f"{el}/floordiv", f"{el}/Cast"], T=T(DT_INT64),
              num_partitions=("i", block_num))
        g.add(f"{el}/Size", "Size", ["Reshape_4"], T=T(DT_INT64), out_type=T(DT_INT32))
        g.const(f"{el}/range/start", 0, DT_INT32)
        g.const(f"{el}/range/delta", 1, DT_INT32)
        g.add(f"{el}/range", "Range", [f"{el}/range/start", f"{el}/Size", f"{el}/range/delta"], Tidx=T(DT_INT32))
        g.add(f"{el}/DynamicPartition_1", "DynamicPartition", [f"{el}/range", f"{el}/Cast"], T=T(DT_INT32),
              num_partitions=("i", block_num))
        gathered = []
        for i in range(block_num):
            nm = f"{el}/GatherV2" + ("" if i == 0 else f"_{i}")
            g.add(nm, "GatherV2", [f"vocab_block_{i}/read", f"{el}/DynamicPartition:{i}", f"{el}/axis"],
                  Tparams=T(DT_FLOAT), Tindices=T(DT_INT64), Taxis=T(DT_INT32), batch_dims=("i", 0))
            gathered.append(nm)
        g.add(f"{el}/DynamicStitch", "DynamicStitch",
              [f"{el}/DynamicPartition_1:{i}" for i in range(block_num)] + gathered, N=("i", block_num),
              T=T(DT_FLOAT))
        params = f"{el}/DynamicStitch"
    # dense FM score
    g.add("Cast", "Cast", ["StringSplit:2"], SrcT=T(DT_INT64), DstT=T(DT_INT32), Truncate=("b", False))
    g.const("Const", [-1], DT_INT32)
    g.const("concat/axis", 0, DT_INT32)
    g.add("concat", "ConcatV2", ["Cast", "Const", "concat/axis"], N=("i", 2), T=T(DT_INT32), Tidx=T(DT_INT32))
    g.const("Slice_2/begin", [0, 1], DT_INT32)
    g.const("Slice_2/size", [-1, -1], DT_INT32)
    g.add("Slice_2", "Slice", [params, "Slice_2/begin", "Slice_2/size"], T=T(DT_FLOAT), Index=T(DT_INT32))
    g.add("Reshape_5", "Reshape", ["Slice_2", "concat"], T=T(DT_FLOAT), Tshape=T(DT_INT32))        # factors
    g.const("Slice_3/begin", [0, 0], DT_INT32)
    g.const("Slice_3/size", [-1, 1], DT_INT32)
    g.add("Slice_3", "Slice", [params, "Slice_3/begin", "Slice_3/size"], T=T(DT_FLOAT), Index=T(DT_INT32))
    g.add("Reshape_6", "Reshape", ["Slice_3", "Cast"], T=T(DT_FLOAT), Tshape=T(DT_INT32))          # biases
    g.const("Const_1", [1], DT_INT32)
    g.const("concat_1/axis", 0, DT_INT32)
    g.add("concat_1", "ConcatV2", ["Cast", "Const_1", "concat_1/axis"], N=("i", 2), T=T(DT_INT32),
          Tidx=T(DT_INT32))
    g.add("Reshape_7", "Reshape", ["SparseToDense_1", "concat_1"], T=T(DT_FLOAT), Tshape=T(DT_INT32))  # fvals
    F = dict(T=T(DT_FLOAT))
    S = dict(T=T(DT_FLOAT), Tidx=T(DT_INT32), keep_dims=("b", False))
    g.add("mul", "Mul", ["Reshape_5", "Reshape_7"], **F)
    g.const("Sum/reduction_indices", 1, DT_INT32)
    g.add("Sum", "Sum", ["mul", "Sum/reduction_indices"], **S)                                       # factor_sum
    g.add("mul_1", "Mul", ["Sum", "Sum"], **F)
    g.const("Sum_1/reduction_indices", [1], DT_INT32)
    g.add("Sum_1", "Sum", ["mul_1", "Sum_1/reduction_indices"], **S)
    g.const("mul_2/x", np.float32(0.5))
    g.add("mul_2", "Mul", ["mul_2/x", "Sum_1"], **F)
    g.add("mul_3", "Mul", ["Reshape_7", "Reshape_7"], **F)
    g.add("mul_4", "Mul", ["mul_3", "Reshape_5"], **F)
    g.add("mul_5", "Mul", ["mul_4", "Reshape_5"], **F)
    g.const("Sum_2/reduction_indices", [1, 2], DT_INT32)
    g.add("Sum_2", "Sum", ["mul_5", "Sum_2/reduction_indices"], **S)
    g.const("mul_6/x", np.float32(0.5))
    g.add("mul_6", "Mul", ["mul_6/x", "Sum_2"], **F)
    g.add("sub", "Sub", ["mul_2", "mul_6"], **F)
    g.add("mul_7", "Mul", ["Reshape_6", "SparseToDense_1"], **F)
    g.const("Sum_3/reduction_indices", [1], DT_INT32)
    g.add("Sum_3", "Sum", ["mul_7", "Sum_3/reduction_indices"], **S)
    out = g.add("add", "AddV2", ["sub", "Sum_3"], **F)
    if global_bias is not None:  # (model extension: the reference has no global bias)
        g.const("global_bias", np.float32(global_bias))
        out = g.add("add_1", "AddV2", ["add", "global_bias"], **F)
    # tf.train.Saver (V2): restore_all assigns every variable from the bundle at save/Const
    names = [f"vocab_block_{i}" for i in range(block_num)]
    g.const("save/filename/input", "model")
    g.add("save/filename", "PlaceholderWithDefault", ["save/filename/input"], dtype=T(DT_STRING), shape=("shape", []))
    g.add("save/Const", "PlaceholderWithDefault", ["save/filename"], dtype=T(DT_STRING), shape=("shape", []))
    g.const("save/SaveV2/tensor_names", names)
    g.const("save/SaveV2/shape_and_slices", [""] * block_num)
    g.add("save/SaveV2", "SaveV2", ["save/Const", "save/SaveV2/tensor_names", "save/SaveV2/shape_and_slices"]
          + names, dtypes=("types", [DT_FLOAT] * block_num))
    g.add("save/control_dependency", "Identity", ["save/Const", "^save/SaveV2"], T=T(DT_STRING))
    g.const("save/RestoreV2/tensor_names", names)
    g.const("save/RestoreV2/shape_and_slices", [""] * block_num)
    g.add("save/RestoreV2", "RestoreV2", ["save/Const", "save/RestoreV2/tensor_names",
                                          "save/RestoreV2/shape_and_slices"], dtypes=("types", [DT_FLOAT] * block_num))
    for i, nm in enumerate(names):
        g.add(f"save/Assign" + ("" if i == 0 else f"_{i}"), "Assign", [nm, f"save/RestoreV2:{i}"], T=T(DT_FLOAT),
              validate_shape=("b", True), use_locking=("b", True))
    g.add("save/restore_all", "NoOp", ["^save/Assign" + ("" if i == 0 else f"_{i}") for i in range(block_num)])
    return g, "test_data:0", out + ":0"


def _tensor_info(name: str, dtype: int) -> bytes:
    """TensorInfo: name = 1, dtype = 2, tensor_shape = 3."""
    return _pb_bytes(1, name.encode()) + _pb_varint(2, dtype) + _pb_bytes(3, shape_proto(None))


def saved_model_proto(graph: GraphBuilder, input_name: str, output_name: str) -> bytes:
    """SavedModel {schema_version = 1, meta_graphs = 2 {meta_info_def = 1, graph_def = 2, saver_def = 3,
    signature_def = 5}}."""
    meta_info = _pb_bytes(4, SERVE_TAG.encode()) + _pb_bytes(5, b"1.15.5")
    saver = (_pb_bytes(1, b"save/Const:0") + _pb_bytes(2, b"save/control_dependency:0")
             + _pb_bytes(3, b"save/restore_all") + _pb_varint(4, 5) + _field5(6) + struct.pack("<f", 10000.0)
             + _pb_varint(7, 2))  # CheckpointFormatVersion V2
    sig = (_map_entry(1, "data_lines", _tensor_info(input_name, DT_STRING))
           + _map_entry(2, "scores", _tensor_info(output_name, DT_FLOAT)) + _pb_bytes(3, PREDICT_METHOD.encode()))
    mg = (_pb_bytes(1, meta_info) + _pb_bytes(2, graph.graph_def()) + _pb_bytes(3, saver)
          + _map_entry(5, SIGNATURE_KEY, sig))
    return _pb_varint(1, 1) + _pb_bytes(2, mg)


def write_saved_model(export_path: str, blocks: list[np.ndarray], vocabulary_size: int, factor_num: int,
                      global_bias: float | None = None) -> list[str]:
    """``saved_model.pb`` + ``variables/variables.{index,data-00000-of-00001}`` (``vocab_block_i``)
    into ``export_path`` (which may already hold other files of the export)."""
    g, inp, out = build_serving_graph(vocabulary_size, len(blocks), factor_num, global_bias)
    os.makedirs(os.path.join(export_path, "variables"), exist_ok=True)
    pb = os.path.join(export_path, "saved_model.pb")
    with open(pb, "wb") as f:
        f.write(saved_model_proto(g, inp, out))
    files = write_bundle(os.path.join(export_path, "variables", "variables"),
                         {f"vocab_block_{i}": np.ascontiguousarray(b, dtype=np.float32) for i, b in enumerate(blocks)})
    return [pb, *files]


# --------------------------------------------------------------------------- independent reader + interpreter
def _decode_shape(buf: bytes):
    f = _parse_pb(buf)
    if f.get(3, [0])[0]:
        return None
    out = []
    for d in f.get(2, []):
        v = _parse_pb(d).get(1, [0])[0]
        out.append(v - (1 << 64) if v >= (1 << 63) else v)
    return out


def _decode_tensor(buf: bytes):
    f = _parse_pb(buf)
    dt = f.get(1, [0])[0]
    shape = _decode_shape(f.get(2, [b""])[0])
    if dt == DT_STRING:
        vals = f.get(8, [])
        return vals[0] if shape == [] else np.array(vals, dtype=object)
    a = np.frombuffer(f.get(4, [b""])[0], dtype=np.dtype(_NP_OF[dt]).newbyteorder("<")).astype(_NP_OF[dt])
    return a.reshape(shape)


def _decode_attr(buf: bytes):
    f = _parse_pb(buf)
    if 2 in f:
        return f[2][0]
    if 3 in f:
        v = f[3][0]
        return v - (1 << 64) if v >= (1 << 63) else v
    if 4 in f:
        return struct.unpack("<f", struct.pack("<I", f[4][0]))[0]
    if 5 in f:
        return bool(f[5][0])
    if 6 in f:
        return f[6][0]
    if 7 in f:
        return _decode_shape(f[7][0])
    if 8 in f:
        return _decode_tensor(f[8][0])
    if 1 in f:
        lst = _parse_pb(f[1][0])
        if 6 in lst:  # packed enum list
            buf6, out, pos = lst[6][0], [], 0
            if isinstance(buf6, int):
                return lst[6]
            while pos < len(buf6):
                v, pos = _read_varint(buf6, pos)
                out.append(v)
            return out
        return []
    return None


def read_saved_model(export_path: str) -> dict:
    """Decode ``saved_model.pb``: {'tags', 'nodes': {name: (op, inputs, attrs)}, 'order', 'saver', 'signatures'}."""
    with open(os.path.join(export_path, "saved_model.pb"), "rb") as f:
        sm = _parse_pb(f.read())
    if sm.get(1, [0])[0] != 1:
        raise ValueError("saved_model_schema_version != 1")
    mg = _parse_pb(sm[2][0])
    info = _parse_pb(mg.get(1, [b""])[0])
    gd = _parse_pb(mg[2][0])
    nodes, order = {}, []
    for nb in gd.get(1, []):
        n = _parse_pb(nb)
        name, op = n[1][0].decode(), n[2][0].decode()
        attrs = {}
        for e in n.get(5, []):
            kv = _parse_pb(e)
            attrs[kv[1][0].decode()] = _decode_attr(kv.get(2, [b""])[0])
        nodes[name] = (op, [i.decode() for i in n.get(3, [])], attrs)
        order.append(name)
    saver = _parse_pb(mg.get(3, [b""])[0])
    sigs = {}
    for e in mg.get(5, []):
        kv = _parse_pb(e)
        s = _parse_pb(kv[2][0])

        def tmap(lst):
            out = {}
            for x in lst:
                y = _parse_pb(x)
                ti = _parse_pb(y[2][0])
                out[y[1][0].decode()] = (ti[1][0].decode(), ti[2][0])
            return out

        sigs[kv[1][0].decode()] = {"inputs": tmap(s.get(1, [])), "outputs": tmap(s.get(2, [])),
                                   "method_name": s[3][0].decode()}
    return {"tags": [t.decode() for t in info.get(4, [])], "nodes": nodes, "order": order,
            "producer": _parse_pb(gd[4][0]).get(1, [0])[0] if 4 in gd else 0,
            "saver": {"filename_tensor_name": saver[1][0].decode(), "restore_op_name": saver[3][0].decode(),
                      "version": saver.get(7, [0])[0]},
            "signatures": sigs}


def _string_split(strings, delim: bytes):
    idx, vals, maxw = [], [], 0
    for i, s in enumerate(strings):
        toks = [t for t in _split_any(s, delim) if t]  # skip_empty
        for j, t in enumerate(toks):
            idx.append((i, j))
            vals.append(t)
        maxw = max(maxw, len(toks))
    return (np.array(idx, dtype=np.int64).reshape(-1, 2), np.array(vals, dtype=object),
            np.array([len(strings), maxw], dtype=np.int64))


def _split_any(s: bytes, delim: bytes):
    """StringSplit: split at ANY of the delimiter's characters."""
    out, cur = [], bytearray()
    for ch in s:
        if ch in delim:
            out.append(bytes(cur))
            cur = bytearray()
        else:
            cur.append(ch)
    out.append(bytes(cur))
    return out


def run_graph(export_path: str, data_lines) -> np.ndarray:
    """Evaluate the exported serving signature on ``data_lines`` with numpy (after running the
    saver's restore op on ``variables/variables``), by the TF ops' documented semantics."""
    sm = read_saved_model(export_path)
    nodes = sm["nodes"]
    sig = sm["signatures"][SIGNATURE_KEY]
    feed_name = sig["inputs"]["data_lines"][0].split(":")[0]
    out_t = sig["outputs"]["scores"][0]
    state: dict[str, np.ndarray] = {}
    restored = read_bundle(os.path.join(export_path, "variables", "variables"))
    cache: dict[str, object] = {}

    def val(ref: str):
        name, _, k = ref.partition(":")
        outs = ev(name)
        return outs[int(k) if k else 0]

    def ev(name: str):
        if name in cache:
            return cache[name]
        op, ins, at = nodes[name]
        data_ins = [i for i in ins if not i.startswith("^")]
        for c in ins:
            if c.startswith("^"):
                ev(c[1:])
        # (Assign takes its variable by reference: the variable is written, not read)
        x = [None if (op == "Assign" and k == 0) else val(i) for k, i in enumerate(data_ins)]
        if op == "Placeholder":
            r = [np.array([s.encode() if isinstance(s, str) else s for s in np.asarray(data_lines, dtype=object)
                           .reshape(-1)], dtype=object)] if name == feed_name else None
        elif op == "PlaceholderWithDefault":
            r = [x[0]]
        elif op == "Const":
            r = [at["value"]]
        elif op == "Identity":
            r = [x[0]]
        elif op == "Reshape":
            r = [np.asarray(x[0]).reshape([int(d) for d in np.asarray(x[1]).reshape(-1)])]
        elif op == "StringSplit":
            r = list(_string_split(list(x[0]), x[1]))
        elif op == "StringToNumber":
            t = _NP_OF[at["out_type"]]
            r = [np.array([t(float(s)) if t is np.float32 else t(int(s)) for s in x[0]], dtype=t)]
        elif op == "Slice":
            b, sz = np.asarray(x[1]), np.asarray(x[2])
            sl = tuple(slice(int(bb), None if int(ss) == -1 else int(bb) + int(ss)) for bb, ss in zip(b, sz))
            r = [np.asarray(x[0])[sl]]
        elif op == "SparseToDense":
            shape = [int(d) for d in x[1]]
            out = np.full(shape, x[3], dtype=np.asarray(x[2]).dtype)
            for (i, j), v in zip(x[0], x[2]):
                out[i, j] = v
            r = [out]
        elif op == "VariableV2":
            r = [state[name]]
        elif op == "Assign":
            want = nodes[data_ins[0]][2].get("shape")
            v = np.asarray(x[1])
            if at.get("validate_shape", True) and want is not None and list(v.shape) != list(want):
                raise ValueError(f"{name}: restored shape {v.shape} != variable shape {want}")
            state[data_ins[0]] = v
            r = [v]
        elif op == "RestoreV2":
            r = [restored[n.decode()] for n in x[1]]
        elif op == "NoOp":
            r = [None]
        elif op == "GatherV2":
            r = [np.take(x[0], np.asarray(x[1]), axis=int(x[2]))]
        elif op == "FloorMod":
            r = [np.mod(x[0], x[1])]
        elif op == "FloorDiv":
            r = [np.floor_divide(x[0], x[1])]
        elif op == "Cast":
            r = [np.asarray(x[0]).astype(_NP_OF[at["DstT"]])]
        elif op == "Size":
            r = [np.int32(np.asarray(x[0]).size)]
        elif op == "Range":
            r = [np.arange(int(x[0]), int(x[1]), int(x[2]), dtype=np.int32)]
        elif op == "DynamicPartition":
            r = [np.asarray(x[0])[np.asarray(x[1]) == p] for p in range(at["num_partitions"])]
        elif op == "DynamicStitch":
            n = at["N"]
            idx, dat = x[:n], x[n:]
            m = max((int(i.max()) for i in idx if i.size), default=-1) + 1
            out = np.zeros((m,) + np.asarray(dat[0]).shape[1:], dtype=np.asarray(dat[0]).dtype)
            for i, d in zip(idx, dat):
                out[np.asarray(i)] = d
            r = [out]
        elif op == "ConcatV2":
            n = at["N"]
            r = [np.concatenate([np.asarray(t).reshape(-1) if np.asarray(t).ndim == 0 else t for t in x[:n]],
                                axis=int(x[n]))]
        elif op == "Mul":
            r = [np.asarray(x[0]) * np.asarray(x[1])]
        elif op == "Sub":
            r = [np.asarray(x[0]) - np.asarray(x[1])]
        elif op == "AddV2":
            r = [np.asarray(x[0]) + np.asarray(x[1])]
        elif op == "Sum":
            ax = tuple(int(a) for a in np.asarray(x[1]).reshape(-1))
            r = [np.asarray(x[0]).sum(axis=ax, keepdims=bool(at.get("keep_dims", False)))]
        else:
            raise NotImplementedError(f"op {op} ({name}) is not interpreted")
        cache[name] = r
        return r

    ev(sm["saver"]["restore_op_name"])   # restore the variables, like the SavedModel loader
    cache.clear()
    return np.asarray(val(out_t), dtype=np.float32)
