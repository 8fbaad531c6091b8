"""Pipeline parallelism: schedule IR, generators, lowering, simulator, runtime."""
from .ir import Action, CommGroup, CommOp, Op, format_compute_grid  # noqa: F401
from .schedules import (SCHEDULES, analytic_bubble, canonical_name, generate, rank_stages,  # noqa: F401
                        stage_to_rank)
from .simulate import check_lowered, simulate  # noqa: F401
from .lower import format_program, lower  # noqa: F401
