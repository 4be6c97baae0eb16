"""circom_cvm_amd: MI355X-native R1CS constraint simplification for circom (--O1/--O2).

The product is librs_simplify.so (HIP kernels for gfx950 + a C++ host orchestrator behind the C ABI
of include/rs_simplify.h).  This package is the thin Python mirror of the reference's
Simplifier -> ConstraintList interface (constraint_list/src/lib.rs:110-202) used by the tests and
the benchmark."""
from .abi import (Engine, Group, Input, Output, PinnedInput, RsError, RsFlags, RsInput, RsOutput, RsStats, check,
                  comm_unique_id, lib, make_flags, simplify_multi)
from .dag import Dag
from .simplifier import ConstraintList, Simplifier

__all__ = ["Engine", "Group", "PinnedInput", "comm_unique_id", "simplify_multi", "Input", "Output", "RsError", "RsFlags", "RsInput", "RsOutput", "RsStats",
           "check", "lib", "make_flags", "Simplifier", "ConstraintList", "Dag"]
