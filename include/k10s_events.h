/*
 * k10s_events.h — event-kind numbering shared by the engine's parity event log and the
 * CPU oracle's event log.  One kind = (destination component, event type) of the reference's
 * dslab handlers, so that two logs can be compared entry by entry.
 *
 * Reference event catalogue: src/core/events.rs:19-244; handlers:
 *   AS  = KubeApiServer::on            src/core/api_server.rs:127-457
 *   PS  = PersistentStorage::on        src/core/persistent_storage.rs:185-490
 *   S   = Scheduler::on                src/core/scheduler/scheduler.rs:382-477
 *   N   = NodeComponent::on            src/core/node_component.rs:178-335
 *   CA  = ClusterAutoscaler::on        src/autoscalers/cluster_autoscaler/cluster_autoscaler.rs:303-334
 *   HPA = HorizontalPodAutoscaler::on  src/autoscalers/horizontal_pod_autoscaler/horizontal_pod_autoscaler.rs:246-257
 *   M   = MetricsCollector::on         src/metrics/collector.rs:410-431
 */
#ifndef K10S_EVENTS_H
#define K10S_EVENTS_H

enum k10s_event_kind {
    K10S_EV_M_POD_METRICS_TICK = 0,   /* RunPodMetricsCollectionCycle        collector.rs:413 */
    K10S_EV_M_GAUGE_TICK = 1,         /* RecordGaugeMetricsCycle (no state)  collector.rs:421 */
    K10S_EV_AS_CREATE_NODE_REQ = 2,   /* CreateNodeRequest     api_server.rs:132 */
    K10S_EV_AS_CREATE_NODE_RESP = 3,  /* CreateNodeResponse    api_server.rs:147 */
    K10S_EV_AS_CREATE_POD_REQ = 4,    /* CreatePodRequest      api_server.rs:151 */
    K10S_EV_AS_ASSIGN_REQ = 5,        /* AssignPodToNodeRequest api_server.rs:163 */
    K10S_EV_AS_ASSIGN_RESP = 6,       /* AssignPodToNodeResponse api_server.rs:194 */
    K10S_EV_AS_POD_NOT_SCHEDULED = 7, /* PodNotScheduled       api_server.rs:219 */
    K10S_EV_AS_POD_STARTED = 8,       /* PodStartedRunning     api_server.rs:233 */
    K10S_EV_AS_POD_FINISHED = 9,      /* PodFinishedRunning    api_server.rs:247 */
    K10S_EV_AS_REMOVE_NODE_REQ = 10,  /* RemoveNodeRequest     api_server.rs:278 */
    K10S_EV_AS_REMOVE_NODE_RESP = 11, /* RemoveNodeResponse    api_server.rs:287 */
    K10S_EV_AS_NODE_REMOVED = 12,     /* NodeRemovedFromCluster api_server.rs:297 */
    K10S_EV_AS_CA_REQ = 13,           /* ClusterAutoscalerRequest api_server.rs:320 */
    K10S_EV_AS_CA_RESP = 14,          /* ClusterAutoscalerResponse api_server.rs:328 */
    K10S_EV_AS_REMOVE_POD_REQ = 15,   /* RemovePodRequest      api_server.rs:342 */
    K10S_EV_AS_REMOVE_POD_RESP = 16,  /* RemovePodResponse     api_server.rs:351 */
    K10S_EV_AS_POD_REMOVED = 17,      /* PodRemovedFromNode    api_server.rs:370 */
    K10S_EV_AS_CREATE_GROUP_REQ = 18, /* CreatePodGroupRequest api_server.rs:405 */
    K10S_EV_PS_CREATE_NODE_REQ = 19,  /* persistent_storage.rs:188 */
    K10S_EV_PS_NODE_ADDED = 20,       /* persistent_storage.rs:197 */
    K10S_EV_PS_CREATE_POD_REQ = 21,   /* persistent_storage.rs:225 */
    K10S_EV_PS_ASSIGN_REQ = 22,       /* persistent_storage.rs:250 */
    K10S_EV_PS_POD_NOT_SCHEDULED = 23,/* persistent_storage.rs:296 */
    K10S_EV_PS_POD_STARTED = 24,      /* persistent_storage.rs:309 */
    K10S_EV_PS_POD_FINISHED = 25,     /* persistent_storage.rs:316 */
    K10S_EV_PS_REMOVE_NODE_REQ = 26,  /* persistent_storage.rs:352 */
    K10S_EV_PS_NODE_REMOVED = 27,     /* persistent_storage.rs:362 */
    K10S_EV_PS_CA_REQ = 28,           /* persistent_storage.rs:381 */
    K10S_EV_PS_REMOVE_POD_REQ = 29,   /* persistent_storage.rs:413 */
    K10S_EV_PS_POD_REMOVED = 30,      /* persistent_storage.rs:460 */
    K10S_EV_S_RUN_CYCLE = 31,         /* RunSchedulingCycle    scheduler.rs:385 */
    K10S_EV_S_FLUSH = 32,             /* FlushUnschedulableQueueLeftover scheduler.rs:388 */
    K10S_EV_S_ADD_NODE = 33,          /* AddNodeToCache        scheduler.rs:391 */
    K10S_EV_S_POD_SCHEDULE_REQ = 34,  /* PodScheduleRequest    scheduler.rs:411 */
    K10S_EV_S_POD_FINISHED = 35,      /* PodFinishedRunning    scheduler.rs:422 */
    K10S_EV_S_REMOVE_NODE = 36,       /* RemoveNodeFromCache   scheduler.rs:441 */
    K10S_EV_S_REMOVE_POD = 37,        /* RemovePodFromCache    scheduler.rs:445 */
    K10S_EV_N_BIND = 38,              /* BindPodToNodeRequest  node_component.rs:181 */
    K10S_EV_N_POD_FINISHED = 39,      /* PodFinishedRunning (self) node_component.rs:227 */
    K10S_EV_N_REMOVE_NODE = 40,       /* RemoveNodeRequest     node_component.rs:247 */
    K10S_EV_N_REMOVE_POD = 41,        /* RemovePodRequest      node_component.rs:275 */
    K10S_EV_CA_TICK = 42,             /* RunClusterAutoscalerCycle cluster_autoscaler.rs:306 */
    K10S_EV_CA_RESP = 43,             /* ClusterAutoscalerResponse cluster_autoscaler.rs:309 */
    K10S_EV_HPA_TICK = 44,            /* RunHorizontalPodAutoscalerCycle horizontal_pod_autoscaler.rs:249 */
    K10S_EV_HPA_REGISTER_GROUP = 45,  /* RegisterPodGroup      horizontal_pod_autoscaler.rs:252 */
    K10S_EV_NUM_KINDS = 46
};

#endif /* K10S_EVENTS_H */
