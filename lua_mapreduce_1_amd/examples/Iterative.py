"""Minimal iterative MapReduce (the control structure of the APRIL-ANN example,
examples/APRIL-ANN/common.lua): state shared through a persistent_table,
finalfn returns "loop" until a stopping criterion holds.

Iteration i: five map jobs each emit ("sum", 2*i); the reduce sums them; the
finalfn appends the total to ``totals`` and stops after 3 iterations."""
from lua_mapreduce_1_amd import persistent_table

CONN = None
DB = "ft_iter"
conf = None


def init(arg):
    global CONN, conf
    if arg:
        CONN = arg[0]
    conf = persistent_table("iter_state", CONN, DB)
    if conf.iterations is None or conf.finished:
        conf.drop()
        conf.set({"iterations": 0, "totals": [], "finished": False})
        conf.update()


def taskfn(emit):
    for i in range(1, 6):
        emit(i, i)


def mapfn(key, value, emit):
    conf.update()
    emit("sum", 2 * (conf.iterations + 1))


def partitionfn(key):
    return 0


def reducefn(key, values, emit):
    emit(sum(values))


def finalfn(pairs):
    conf.update()
    total = None
    for k, v in pairs:
        total = v[0]
    conf.set({"iterations": conf.iterations + 1, "totals": list(conf.totals) + [total]})
    if conf.iterations >= 3:
        conf.set({"finished": True})
        conf.update()
        return True
    conf.update()
    return "loop"
