"""CPU: the lazy info dict of HeliVecEnv.step() (heligym_amd.vector.LazyInfo) -- keys present at
once, each value computed on first read only, a read after the step's buffers were reused raises,
and it compares like the plain dict of its values."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "heli-gym_amd"))

from heligym_amd import _abi  # noqa: E402
from heligym_amd.vector import LazyInfo  # noqa: E402


def make(valid_flag, calls):
    def th(key, value):
        def f(info):
            calls.append(key)
            return value
        return f

    def pair(info):   # two keys from one computation, cached on the info object
        r = getattr(info, "_pair", None)
        if r is None:
            calls.append("pair")
            r = info._pair = (1, 2)
        return r
    thunks = {"a": th("a", 10), "b": th("b", 20), "p0": lambda i: pair(i)[0], "p1": lambda i: pair(i)[1]}
    return LazyInfo(thunks, lambda: valid_flag[0]), thunks


def test_lazy_fields_computed_once_on_first_read():
    calls, valid = [], [True]
    info, thunks = make(valid, calls)
    assert set(info) == {"a", "b", "p0", "p1"} and len(info) == 4 and "a" in info
    assert calls == []
    assert info["a"] == 10 and info["a"] == 10
    assert calls == ["a"]
    assert info["p1"] == 2 and info["p0"] == 1
    assert calls == ["a", "pair"]            # one computation for both keys
    assert info.get("b") == 20 and info.get("zz", 5) == 5
    assert calls == ["a", "pair", "b"]
    other, _ = make(valid, [])
    assert other == info == {"a": 10, "b": 20, "p0": 1, "p1": 2}
    assert dict(info.items()) == {"a": 10, "b": 20, "p0": 1, "p1": 2}
    # the shared thunk table is not consumed by one step's info
    assert set(thunks) == {"a", "b", "p0", "p1"}


def test_read_after_reuse_raises_but_cached_values_stay():
    calls, valid = [], [True]
    info, _ = make(valid, calls)
    assert info["a"] == 10
    valid[0] = False
    assert info["a"] == 10                   # already read: still served
    with pytest.raises(_abi.HeliGymError):
        info["b"]
    with pytest.raises(_abi.HeliGymError):
        info.copy()


def test_mutating_reads_never_return_placeholders():
    """pop / popitem / setdefault / update / pickling go through the lazy read like __getitem__
    (dict's own versions would hand out the None placeholder of an unread field)."""
    import copy
    import pickle
    calls, valid = [], [True]
    info, _ = make(valid, calls)
    assert info.pop("b") == 20 and "b" not in info and calls == ["b"]
    assert info.pop("b", 7) == 7
    with pytest.raises(KeyError):
        info.pop("b")
    assert info.setdefault("a", 99) == 10 and info.setdefault("new", 3) == 3 and info["new"] == 3
    k, v = info.popitem()
    assert (k, v) == ("new", 3)
    info.update(p0=-1)
    assert info["p0"] == -1 and "p0" not in info._pending
    assert pickle.loads(pickle.dumps(info)) == {"a": 10, "p0": -1, "p1": 2}
    assert copy.deepcopy(info) == {"a": 10, "p0": -1, "p1": 2}
    valid[0] = False
    info2, _ = make(valid, [])
    with pytest.raises(_abi.HeliGymError):
        info2.pop("a")
    with pytest.raises(_abi.HeliGymError):
        info2.setdefault("a")
