"""Archived round 5: the Python side of the 11-bit u32 sort (ops/primitives.py), removed with
csrc/hip/sort11.hip after it measured 17-35 ms vs 10.0 ms per TeraSort step (profiles/r5/terasort/)."""
# flake8: noqa
_SORT11_WS: dict = {}


def _sort_keys32_11(k32: torch.Tensor):
    """sort_keys32 in THREE onesweep passes of 11 + 11 + 10 bits
    (csrc/hip/sort11.hip; ``MR_SORT32_DIGIT_BITS=11``): its own histogram
    pass ([3][2048] bins), 2048 look-back granules per tile."""
    n = k32.numel()
    d = k32.device
    s = _hip.stream(d)
    lib = _hip.lib()
    tiles = int(lib.mr_sort11_tiles(n))
    ws = _SORT11_WS.get(d)
    if ws is None or ws["tiles"] < tiles:
        ws = {"tiles": tiles, "granules": torch.zeros(tiles * 2048, dtype=torch.int64, device=d),
              "small": torch.zeros(3 * 2048 + 64 + 1, dtype=torch.int32, device=d)}
        _SORT11_WS[d] = ws
    small = ws["small"]
    small.zero_()
    _hip.call("mr_hist11", _hip.ptr(k32), n, _hip.ptr(small[:3 * 2048]), s)
    kbuf = [torch.empty(n, dtype=torch.int32, device=d) for _ in range(2)]
    pbuf = [torch.empty(n, dtype=torch.int32, device=d) for _ in range(2)]
    kin, pin = k32.contiguous(), None
    for pass_id, (shift, mask) in enumerate(((0, 0x7FF), (11, 0x7FF), (22, 0x3FF))):
        _EPOCH[0] = (_EPOCH[0] + 1) & 0xFFFFFF or 1
        kout = kbuf[0] if kin is not kbuf[0] else kbuf[1]
        pout = pbuf[0] if pin is not pbuf[0] else pbuf[1]
        _hip.call("mr_radix_onesweep11", _hip.ptr(kin), _hip.ptr(pin), _hip.ptr(kout), _hip.ptr(pout), n, shift, mask,
                  _hip.ptr(small[pass_id * 2048:(pass_id + 1) * 2048]), _hip.ptr(ws["granules"]),
                  _hip.ptr(small[3 * 2048 + pass_id:]), _EPOCH[0], _hip.ptr(small[3 * 2048 + 64:]),
                  1 if pin is None else 0, s)
        kin, pin = kout, pout
    _SORT11_ERR[d] = small[3 * 2048 + 64:]
    _LAST11[d] = True
    return pin, kin


_SORT11_ERR: dict = {}
_LAST11: dict = {}  # device -> the last u32 sort took the 11-bit passes (sort_error reads its error word)
