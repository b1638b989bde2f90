from tilelang.ir import expr as E
from tilelang.ir.dtypes import float16, float32


def test_constant_folding_and_identities():
    x = E.Var("x")
    assert E.as_int(E.const(3) * 4 + 1) == 13
    assert (x + 0) is x
    assert (x * 1) is x
    assert E.as_int(x * 0) == 0
    e = (x + 1) * 128 - x * 128
    assert E.as_int(e) == 128
    e2 = (x + 7) - (x + 2)
    assert E.as_int(e2) == 5


def test_type_promotion():
    h = E.Var("h", float16)
    f = E.Var("f", float32)
    assert (h + 1).dtype == float16
    assert (h + f).dtype == float32
    assert (E.Var("i") + 1.5).dtype == float32


def test_evaluate_matches_c_semantics():
    x = E.Var("x")
    env = {x: 17}
    assert E.evaluate(x // 4, env) == 4
    assert E.evaluate(x % 4, env) == 1
    fn = E.compile_py(x * 3 + (x >> 1), [x])
    assert fn(10) == 35


def test_modular_analysis():
    t = E.Var("t")
    assert E.divisible_by(t * 8 + 16, 8)
    assert not E.divisible_by(t * 8 + 4, 8)
    assert E.divisible_by(((t // 16) % 4) * 4, 4)


def test_substitute_and_structural_equal():
    x, y = E.Var("x"), E.Var("y")
    e = x * 2 + y
    e2 = E.substitute(e, {x: E.const(3)})
    assert E.structural_equal(e2, 6 + y) or E.structural_equal(e2, y + 6)
