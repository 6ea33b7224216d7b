from .tasks import (
    AVAILABLE_TASK_NAMES,
    TASK_REGISTRY,
    TaskConfig,
    TaskStrategy,
    compute_predictions_for_tasks,
    compute_probabilities_for_tasks,
    create_loss_functions,
    get_strategy,
    get_task,
    get_tasks,
    register_task,
)

__all__ = [
    "AVAILABLE_TASK_NAMES", "TASK_REGISTRY", "TaskConfig", "TaskStrategy", "compute_predictions_for_tasks",
    "compute_probabilities_for_tasks", "create_loss_functions", "get_strategy", "get_task", "get_tasks",
    "register_task",
]
