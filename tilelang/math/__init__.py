"""Small integer helpers (reference: tilelang/math/__init__.py)."""


def next_power_of_2(x: int) -> int:
    """Smallest power of two >= x (1 for x <= 1)."""
    x = int(x)
    return 1 if x <= 1 else 1 << (x - 1).bit_length()


def cdiv(a: int, b: int) -> int:
    """Ceiling division of Python ints (use ``T.ceildiv`` inside kernels)."""
    return -(-int(a) // int(b))


def prev_power_of_2(x: int) -> int:
    x = int(x)
    return 0 if x < 1 else 1 << (x.bit_length() - 1)
