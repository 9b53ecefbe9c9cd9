"""Predictors that map symbols themselves (SURVEY.md §8(b) "arbitrary Predictor
subclasses with custom symbol_to_range").  ``make(Predictor, CDFPredictor)``
builds them over either the reference's base classes (tools/gen_golden_custom.py,
which records what the reference coder does with them) or lac_amd.coder's
(tests), so both sides run the same mapping code."""
import bisect


def make(Predictor, CDFPredictor):
    class Fixed(Predictor):
        """Ranges from a fixed list, whatever the interval width (the shape of the
        reference's ModifiedMarkov, arith_code.py:468-507)."""

        def __init__(self, edges):
            self.n = len(edges)
            self.edges = list(edges)

        def val_to_symbol(self, v, denom):
            return bisect.bisect_right(self.edges, v)

        def symbol_to_range(self, s, denom):
            return (self.edges[s - 1] if s > 0 else 0), self.edges[s]

        def copy(self):
            return Fixed(self.edges)

    class FloorCDF(CDFPredictor):
        """A CDF table coded with the floor mapping instead of CDFPredictor's ceil."""

        def symbol_to_range(self, s, denom):
            if s < 0 or s >= len(self.dist):
                raise AssertionError("unknown symbol", s)
            T = self.dist[-1]
            return ((self.dist[s - 1] if s > 0 else 0) * denom) // T, (self.dist[s] * denom) // T

        def val_to_symbol(self, v, denom):
            T = self.dist[-1]
            return bisect.bisect_right([(c * denom) // T for c in self.dist], v)

    class Counting(Predictor):
        """Adaptive counts, floor-scaled into the interval by its own rule."""

        def __init__(self, n, counts=None):
            self.n = n
            self.counts = list(counts) if counts else [1] * n

        def _edges(self, denom):
            tot, c, out = sum(self.counts), 0, []
            for k in self.counts:
                c += k
                out.append((c * denom) // tot)
            return out

        def val_to_symbol(self, v, denom):
            return bisect.bisect_right(self._edges(denom), v)

        def symbol_to_range(self, s, denom):
            e = self._edges(denom)
            return (e[s - 1] if s > 0 else 0), e[s]

        def accept(self, s):
            self.counts[s] += 3

        def copy(self):
            return Counting(self.n, self.counts)

    return Fixed, FloorCDF, Counting


def build(kind, Fixed, FloorCDF, Counting, params):
    if kind == "fixed":
        return Fixed(params)
    if kind == "floorcdf":
        return FloorCDF(params)
    return Counting(params)
