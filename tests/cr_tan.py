"""Correctly rounded fp64 tan by 70-digit Decimal arithmetic (test infrastructure).

float(Decimal) rounds correctly, so cr_tan(x) is the fp64 value nearest the
exact tan of the double x.  Used to pin csrc/sk_tan_cr.hpp and to classify the
probe boards where glibc's math.tan (the reference's) is not correctly rounded.
"""
from decimal import Decimal, localcontext

_PI = Decimal("3.14159265358979323846264338327950288419716939937510582097494459230781640628620899862803482534211706798")
_EPS = Decimal(10) ** -72


def cr_tan(x):
    with localcontext() as ctx:
        ctx.prec = 80
        d = Decimal(float(x))
        k = (d / (_PI / 2)).to_integral_value()
        r = d - k * (_PI / 2)
        r2 = r * r
        s, term, i = Decimal(0), r, 1
        while abs(term) > _EPS:
            s += term
            term = -term * r2 / ((2 * i) * (2 * i + 1))
            i += 1
        c, term, i = Decimal(0), Decimal(1), 1
        while abs(term) > _EPS:
            c += term
            term = -term * r2 / ((2 * i - 1) * (2 * i))
            i += 1
        t = -c / s if int(k) % 2 else s / c
        return float(t)
