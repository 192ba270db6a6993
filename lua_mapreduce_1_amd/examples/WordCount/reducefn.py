"""WordCount reducefn (reference: examples/WordCount/reducefn.lua): sum, also
the combiner, with the associative/commutative/idempotent flags."""


def init(arg):
    pass


def reducefn(key, values, emit):
    emit(sum(values))


combinerfn = reducefn
device_reduce = "sum"
associative_reducer = True
commutative_reducer = True
idempotent_reducer = True
