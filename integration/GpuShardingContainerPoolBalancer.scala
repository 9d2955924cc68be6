/*
 * Drop-in LoadBalancerProvider for the MI355X engine (SOURCE ONLY: this image has no JDK/scalac, see DESIGN.md).
 *
 * A maintainer adds this file to core/controller/src/main/scala/org/apache/openwhisk/core/loadBalancer/ and selects
 * it with   whisk.spi.LoadBalancerProvider = org.apache.openwhisk.core.loadBalancer.GpuShardingContainerPoolBalancer
 * (common/scala/src/main/resources/reference.conf:26, or CONFIG_whisk_spi_LoadBalancerProvider).
 *
 * Everything except the scheduling state stays as in ShardingContainerPoolBalancer (SCPB): CommonLoadBalancer keeps
 * activation bookkeeping, the Kafka send, the ack feed and processCompletion; the monitor actor keeps forwarding
 * CurrentInvokerPoolState and cluster membership.  publish() enqueues into a single batching thread that owns the
 * native context (single writer, owgs.h "Threading"), which calls owgs_publish_batch and completes the promises in
 * stream order; releaseInvoker() enqueues into the same thread (owgs_release_batch).
 */
package org.apache.openwhisk.core.loadBalancer

import java.util.concurrent.{ArrayBlockingQueue, TimeUnit}

import akka.actor.{Actor, ActorRef, ActorRefFactory, ActorSystem, Props}
import akka.stream.ActorMaterializer
import org.apache.kafka.clients.producer.RecordMetadata
import org.apache.openwhisk.common._
import org.apache.openwhisk.core.WhiskConfig
import org.apache.openwhisk.core.WhiskConfig._
import org.apache.openwhisk.core.connector._
import org.apache.openwhisk.core.entity._
import org.apache.openwhisk.spi.SpiLoader

import scala.collection.mutable
import scala.concurrent.{Future, Promise}

/** JNI surface of libowgs.so (include/owgs.h); implemented by integration/owgs_jni.c. */
object OwgsNative {
  System.loadLibrary("owgs_jni")
  @native def create(managedFraction: Double, blackboxFraction: Double, minMemoryBytes: Long, clusterSize: Int,
                     device: Int, rngSeed: Long): Long
  @native def destroy(ctx: Long): Unit
  @native def updateInvokers(ctx: Long, ids: Array[Int], userMemoryBytes: Array[Long], status: Array[Byte]): Int
  @native def updateCluster(ctx: Long, size: Int): Int
  @native def registerAction(ctx: Long, namespace: String, path: String, key: String, memMb: Int, maxConc: Int,
                             blackbox: Boolean): Int
  @native def publishBatch(ctx: Long, actions: Array[Int], seq: Array[Long], n: Int, outInvoker: Array[Int],
                           outFlags: Array[Byte]): Int
  @native def releaseBatch(ctx: Long, invokers: Array[Int], actions: Array[Int], n: Int, outFlags: Array[Byte]): Int
  @native def lastError(ctx: Long): String
}

class GpuShardingContainerPoolBalancer(config: WhiskConfig,
                                       controllerInstance: ControllerInstanceId,
                                       feedFactory: FeedFactory,
                                       val invokerPoolFactory: InvokerPoolFactory,
                                       implicit val messagingProvider: MessagingProvider =
                                         SpiLoader.get[MessagingProvider])(implicit actorSystem: ActorSystem,
                                                                           logging: Logging,
                                                                           materializer: ActorMaterializer)
    extends CommonLoadBalancer(config, feedFactory, controllerInstance) {

  private val ctx = OwgsNative.create(lbConfig.managedFraction, lbConfig.blackboxFraction,
    MemoryLimit.MIN_MEMORY.toBytes, 1, 0, 0x0F15C005L)

  // (invoking namespace, fqn@version) -> native action handle (registered once); fqn@version -> a handle of that
  // action for releases (a release only needs the NestedSemaphore key and the limits, NS:98-113)
  private val handles = mutable.HashMap.empty[(String, String), Int]
  private val byKey = mutable.HashMap.empty[String, Int]
  @volatile private var invokerList: IndexedSeq[InvokerHealth] = IndexedSeq.empty
  @volatile private var _clusterSize = 1

  private sealed trait Job
  private case class Pub(action: ExecutableWhiskActionMetaData, msg: ActivationMessage, seq: Long,
                         p: Promise[Option[(InvokerInstanceId, Boolean)]]) extends Job
  private case class Rel(invoker: InvokerInstanceId, entry: ActivationEntry) extends Job
  private case class Inv(state: IndexedSeq[InvokerHealth]) extends Job
  private case class Clu(size: Int) extends Job

  private val queue = new ArrayBlockingQueue[Job](1 << 16)
  private var seqNo = 0L

  /** The single writer of the native context: drains the queue in batches (stream order is the sequential order). */
  private val batcher = new Thread(() => {
    val jobs = new java.util.ArrayList[Job](4096)
    while (true) {
      val first = queue.poll(1, TimeUnit.MILLISECONDS)
      if (first != null) {
        jobs.add(first)
        queue.drainTo(jobs, 4095)
        var i = 0
        while (i < jobs.size) {
          jobs.get(i) match {
            case Inv(s) =>
              OwgsNative.updateInvokers(ctx, s.map(_.id.toInt).toArray, s.map(_.id.userMemory.toBytes).toArray,
                s.map(h => statusCode(h.status)).toArray)
              i += 1
            case Clu(n) => OwgsNative.updateCluster(ctx, n); i += 1
            case _ =>
              // maximal run of releases followed by publishes: one native call each, order preserved
              val rels = mutable.ArrayBuffer.empty[Rel]
              while (i < jobs.size && jobs.get(i).isInstanceOf[Rel]) { rels += jobs.get(i).asInstanceOf[Rel]; i += 1 }
              if (rels.nonEmpty) {
                val inv = rels.map(_.invoker.toInt).toArray
                val act = rels.map(r => byKey(r.entry.fullyQualifiedEntityName.asString)).toArray
                OwgsNative.releaseBatch(ctx, inv, act, inv.length, new Array[Byte](inv.length))
              }
              val pubs = mutable.ArrayBuffer.empty[Pub]
              while (i < jobs.size && jobs.get(i).isInstanceOf[Pub]) { pubs += jobs.get(i).asInstanceOf[Pub]; i += 1 }
              if (pubs.nonEmpty) {
                val act = pubs.map(p => handleOf(p.msg.user.namespace.name.asString, p.action.fullyQualifiedName(true),
                  p.action.limits.memory.megabytes, p.action.limits.concurrency.maxConcurrent, p.action.exec.pull)).toArray
                val out = new Array[Int](act.length)
                val flags = new Array[Byte](act.length)
                OwgsNative.publishBatch(ctx, act, pubs.map(_.seq).toArray, act.length, out, flags)
                pubs.zipWithIndex.foreach { case (p, k) =>
                  val r =
                    if (out(k) >= 0) Some((InvokerInstanceId(out(k), userMemory = invokerMemory(out(k))), (flags(k) & 1) != 0))
                    else None // -1: no invokers; -2: the reference's schedule() would have thrown
                  p.p.success(r)
                }
              }
          }
        }
        jobs.clear()
      }
    }
  }, "owgs-batcher")
  batcher.setDaemon(true)
  batcher.start()

  private def statusCode(s: InvokerState): Byte = s match {
    case InvokerState.Healthy      => 0
    case InvokerState.Unhealthy    => 1
    case InvokerState.Unresponsive => 2
    case InvokerState.Offline      => 3
  }

  private def invokerMemory(id: Int): ByteSize = invokerList.find(_.id.toInt == id).map(_.id.userMemory).getOrElse(0.B)

  private def handleOf(ns: String, fqn: FullyQualifiedEntityName, memMb: Int, maxConc: Int, blackbox: Boolean): Int =
    handles.getOrElseUpdate((ns, fqn.asString), {
      val h = OwgsNative.registerAction(ctx, ns, fqn.copy(version = None).asString, fqn.asString, memMb, maxConc,
        blackbox)
      byKey.getOrElseUpdate(fqn.asString, h)
      h
    })

  // state updates go through the batching thread too, so they are serialized with publishes exactly like the
  // reference's monitor actor serializes updateInvokers / updateCluster (SCPB:210-250)
  private val monitor = actorSystem.actorOf(Props(new Actor {
    private var members = Set.empty[akka.cluster.Member]
    override def preStart(): Unit =
      if (actorSystem.settings.config.getStringList("akka.cluster.seed-nodes").size > 0)
        akka.cluster.Cluster(actorSystem)
          .subscribe(self, classOf[akka.cluster.ClusterEvent.MemberEvent], classOf[akka.cluster.ClusterEvent.ReachabilityEvent])
    override def receive: Receive = {
      case CurrentInvokerPoolState(newState) => invokerList = newState; queue.put(Inv(newState))
      case akka.cluster.ClusterEvent.CurrentClusterState(ms, _, _, _, _) =>
        members = ms.filter(_.status == akka.cluster.MemberStatus.Up)
        _clusterSize = math.max(1, members.size); queue.put(Clu(members.size))
      case e: akka.cluster.ClusterEvent.ClusterDomainEvent =>
        members = e match {
          case akka.cluster.ClusterEvent.MemberUp(m)          => members + m
          case akka.cluster.ClusterEvent.ReachableMember(m)   => members + m
          case akka.cluster.ClusterEvent.MemberRemoved(m, _)  => members - m
          case akka.cluster.ClusterEvent.UnreachableMember(m) => members - m
          case _                                             => members
        }
        _clusterSize = math.max(1, members.size); queue.put(Clu(members.size))
    }
  }))

  override def invokerHealth(): Future[IndexedSeq[InvokerHealth]] = Future.successful(invokerList)
  override def clusterSize: Int = _clusterSize

  /** SCPB:257-317 with the schedule() half (SCPB:260-290) executed natively in batches. */
  override def publish(action: ExecutableWhiskActionMetaData, msg: ActivationMessage)(
    implicit transid: TransactionId): Future[Future[Either[ActivationId, WhiskActivation]]] = {
    val p = Promise[Option[(InvokerInstanceId, Boolean)]]()
    val s = synchronized { seqNo += 1; seqNo }
    queue.put(Pub(action, msg, s, p))
    p.future.flatMap {
      case Some((invoker, overload)) =>
        if (overload)
          MetricEmitter.emitCounterMetric(
            if (action.exec.pull) LoggingMarkers.BLACKBOX_SYSTEM_OVERLOAD else LoggingMarkers.MANAGED_SYSTEM_OVERLOAD)
        val activationResult = setupActivation(msg, action, invoker)
        sendActivationToInvoker(messageProducer, msg, invoker).map(_ => activationResult)
      case None => Future.failed(LoadBalancerException("No invokers available"))
    }
  }

  override val invokerPool: ActorRef = invokerPoolFactory.createInvokerPool(
    actorSystem, messagingProvider, messageProducer, sendActivationToInvoker, Some(monitor))

  /** SCPB:327-331: releaseConcurrent through the native context. */
  override protected def releaseInvoker(invoker: InvokerInstanceId, entry: ActivationEntry): Unit =
    queue.put(Rel(invoker, entry))
}

object GpuShardingContainerPoolBalancer extends LoadBalancerProvider {
  override def instance(whiskConfig: WhiskConfig, instance: ControllerInstanceId)(
    implicit actorSystem: ActorSystem, logging: Logging, materializer: ActorMaterializer): LoadBalancer = {
    // the same invoker-supervision wiring the reference provider builds (SCPB:341-358): health pings from the
    // "health" topic drive InvokerPool, which reports CurrentInvokerPoolState to our monitor actor
    val pools = new InvokerPoolFactory {
      override def createInvokerPool(f: ActorRefFactory, mp: MessagingProvider, producer: MessageProducer,
                                     send: (MessageProducer, ActivationMessage, InvokerInstanceId) => Future[RecordMetadata],
                                     monitor: Option[ActorRef]): ActorRef = {
        InvokerPool.prepare(instance, WhiskEntityStore.datastore())
        val healthFeed = mp.getConsumer(whiskConfig, s"health${instance.asString}", "health", maxPeek = 128)
        f.actorOf(InvokerPool.props((af, i) => af.actorOf(InvokerActor.props(i, instance)),
          (m, i) => send(producer, m, i), healthFeed, monitor))
      }
    }
    new GpuShardingContainerPoolBalancer(whiskConfig, instance, createFeedFactory(whiskConfig, instance), pools)
  }

  def requiredProperties: Map[String, String] = kafkaHosts
}
