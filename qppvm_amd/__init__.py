"""qppvm_amd: MI355X-native batched whole-body-QP engine (QPPVM torque solve)."""
from .problem import (QPPVMProblem, SELECT_SUBTASK, SELECT_TASK, WEIGHT_IDENTITY, WEIGHT_INERTIA,
                      STATUS_OK, STATUS_MAXITER, STATUS_INFEASIBLE, STATUS_NUMERICAL)
