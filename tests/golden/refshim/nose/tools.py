"""nose.tools stand-in for running the reference's own tests in the build container (fixture capture only)."""
import unittest
_tc = unittest.TestCase()
assert_raises = _tc.assertRaises
assert_sequence_equal = _tc.assertSequenceEqual
