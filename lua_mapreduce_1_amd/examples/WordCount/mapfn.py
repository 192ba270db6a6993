"""WordCount mapfn (reference: examples/WordCount/mapfn.lua): whitespace tokens.

``device_mapfn`` is the GPU form: the file is staged to HBM and every token is
counted by the fused tokenizer/combiner kernel (csrc/hip/wordcount3.hip)."""
from lua_mapreduce_1_amd.ops import io as _io


def init(arg):
    pass


def mapfn(key, value, emit):
    with open(value, "rb") as f:
        for line in f:
            for w in line.split():
                emit(w.decode("utf-8", "surrogateescape"), 1)


def device_mapfn(key, value, emit):
    # value: a file path (server/worker jobs) or the staged input tensor (SPMD engine)
    emit.words(value if hasattr(value, "data_ptr") else _io.load_file(value, emit.device))
