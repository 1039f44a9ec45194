"""``apps.kubedl.io/v1alpha1`` -- the Cron API (reference: ``api/v1alpha1/``)."""
from .groupversion import (  # noqa: F401
    CRON_GVK,
    CRON_GVR,
    GROUP,
    GROUP_VERSION,
    KIND_CRON,
    LABEL_CRON_NAME,
    LABEL_PREFIX_KUBEDL,
    RESOURCE_CRONS,
    VERSION,
)
from .types import (  # noqa: F401
    CONCURRENCY_POLICIES,
    ConcurrentPolicyAllow,
    ConcurrentPolicyForbid,
    ConcurrentPolicyReplace,
    Cron,
    CronHistory,
    CronSpec,
    CronStatus,
    CronTemplateSpec,
    JobFailed,
    JobRunning,
    JobSucceeded,
    ObjectReference,
    TypedLocalObjectReference,
    new_cron,
)
