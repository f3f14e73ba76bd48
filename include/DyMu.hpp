// DyMu.hpp -- PathPlanning_lib::DyMuPathPlanner, the global-layer surface of
// the reference class (src/DyMu.hpp:397-609) re-implemented over row-major
// SoA arrays, with the total-cost propagation delegated to the MI355X engine
// through the C-ABI in dymu_fim.h.
//
// Same method names, argument meaning and return values as the reference for
// the hot path and its two neighbours (cost-map ingestion, path extraction):
//   initGlobalLayer      src/DyMu_GlobalPathPlanning.cpp:39-104
//   setCostMap           :109-126
//   computeCostMap       :145-181 (+ :186-308, quirks Q1-Q4 of SURVEY s8(a))
//   setGoal              :322-357
//   computeTotalCostMap  :364-408
//   computeEntireTotalCostMap :443-468
//   getPath / computeGlobalPath :589-662 (+ :666-784)
//   getTotalCostMatrix, getGlobalCostMatrix, getHazardDensityMatrix,
//   getTrafficabilityMatrix, getTotalCost, getLocomotionMode  :788-890
//   local layer (src/DyMu_LocalPathRepairing.cpp, csrc/local_layer.cpp):
//   computeLocalPlanning, repairPath, evaluatePath, expandRisk,
//   computeLocalPropagation, getLocalPath, computeLocalWaypointGDM,
//   getRiskMatrix, getDeviationMatrix, getReconnectingIndex, getLocalNode,
//   subdivideGlobalNode, getTotalCost(localNode)
// Differences a caller can see:
//   * nodes are SoA arrays, not heap records: getGlobalNode /
//     getNearestGlobalNode / getLocalNode return snapshots (std::optional for
//     the reference's NULL), node-taking methods take grid indices or a
//     snapshot; CoRa (cost-ratio learning) is not part of this library.
//   * computeTotalCostMap stops like the reference once the start and its nb4
//     are final: CLOSED cells hold their converged values, the
//     narrow band the reference's tentative values (replayed on the host from
//     the CLOSED values), every other cell +inf; ties between equal total
//     costs follow the reference's insertion order, rebuilt from the values
//     (csrc/pop_order.hpp), and so does the band list.
//   * the node-pointer members are accessors returning snapshots:
//     globalNarrowband(), globalPropagatedNodes(), globalGoal(), localAgent(),
//     localNarrowband(), localExpandableObstacles(), localPropagatedNodes(); a
//     node's public `state` is written through setGlobalNodeState.  The per-node
//     steps of the loops the library runs whole are there too, by grid index or
//     snapshot (propagateGlobalNode, maxRiskNode, propagateRisk,
//     propagateLocalNode, minCostLocalNode x2), so a caller can drive the
//     reference's loops itself.  setHorizonCost (src/DyMu.hpp:555) is declared
//     but defined nowhere in the reference (a caller cannot link it there); it
//     is not provided.
//   * a start or goal on the border returns false instead of dereferencing
//     NULL (reference :416-417, :430-431).
#pragma once

#include <cstdint>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <vector>

#include "dymu_base.hpp"
#include "dymu_fim.h"

namespace PathPlanning_lib {

enum node_state { OPEN, CLOSED };

enum repairingAproach {
  CONSERVATIVE,  // Hazard Avoidance - FM*
  SWEEPING       // multiBiFM*
};

// Snapshot of a global node (the reference's globalNode, src/DyMu.hpp:69-108,
// without the neighbour pointer lists and the local map).
struct globalNode {
  base::Pose2D pose;        // grid indices (i, j)
  base::Pose2D world_pose;  // i * res, j * res
  double elevation = 0.0, slope = 0.0;
  node_state state = OPEN;
  bool isObstacle = false;
  bool hasLocalMap = false;
  double raw_cost = 0.0, cost = 0.0, hazard_density = 0.0, trafficability = 1.0;
  double total_cost = 0.0;
  unsigned terrain = 0;
  std::string nodeLocMode = "DONT_CARE";
};

// Snapshot of a local-layer sub-cell (the reference's localNode,
// src/DyMu.hpp:42-67, without nb4List).  id names the sub-cell for the
// node-taking methods below.
struct localNode {
  base::Pose2D pose;         // sub-cell indices inside the parent global node
  base::Pose2D world_pose;   // global_pose / global_res
  base::Pose2D parent_pose;  // parent global node (grid indices)
  base::Pose2D global_pose;  // in global units
  double deviation = 0.0, total_cost = 0.0, cost = 0.0, risk = 0.0;
  node_state state = OPEN;
  bool isObstacle = false;
  uint64_t id = 0;
};

struct LocalLayer;  // csrc/local_layer.hpp
struct PathIndex;   // csrc/local_layer.hpp
struct TieGuard;    // csrc/pop_order.hpp

class DyMuPathPlanner {
 public:
  // -- public state kept from the reference (src/DyMu.hpp:444-467) --
  std::vector<base::Waypoint> current_path;  // the last computed path
  std::vector<double> cost_lutable;          // cost LUT (computeCostMap)
  double remaining_total_cost = 0.0;
  int reconnecting_index = 0;

  DyMuPathPlanner(double risk_distance, double reconnect_distance, double risk_ratio,
                  repairingAproach input_approach);
  ~DyMuPathPlanner();
  DyMuPathPlanner(const DyMuPathPlanner&) = delete;
  DyMuPathPlanner& operator=(const DyMuPathPlanner&) = delete;

  bool initGlobalLayer(double globalres, double localres, unsigned num_nodes_X,
                       unsigned num_nodes_Y, std::vector<double> offset);
  bool setCostMap(std::vector<std::vector<double>> cost_map);
  bool computeCostMap(std::vector<double> cost_data, std::vector<double> slope_values,
                      std::vector<std::string> locomotionModes,
                      std::vector<std::vector<double>> elevation,
                      std::vector<std::vector<double>> terrainMap);
  // the same from row-major nx*ny arrays (the flat C-ABI's path: no per-row copies)
  bool computeCostMap(const std::vector<double>& cost_data,
                      const std::vector<double>& slope_values,
                      const std::vector<std::string>& locomotionModes, const double* elevation,
                      const double* terrainMap);

  // the per-node steps of computeCostMap (src/DyMu.hpp:493-497), by grid index
  void calculateSlope(unsigned i, unsigned j);
  void calculateNominalCost(unsigned i, unsigned j, int range, int numLocs);
  void smoothCost(unsigned i, unsigned j);

  bool setGoal(base::Waypoint wGoal);
  bool computeTotalCostMap(base::Waypoint wPos);
  bool computeEntireTotalCostMap();

  std::vector<base::Waypoint> getPath(base::Waypoint wPos);
  bool computeGlobalPath(base::Waypoint wPos);
  base::Waypoint computeNextGlobalWaypoint(base::Waypoint& wPos, double tau);
  double interpolate(double a, double b, double g00, double g01, double g10, double g11);

  std::string getLocomotionMode(base::Waypoint wPos);
  std::vector<std::vector<double>> getTotalCostMatrix();
  std::vector<std::vector<double>> getGlobalCostMatrix();
  std::vector<std::vector<double>> getHazardDensityMatrix();
  std::vector<std::vector<double>> getTrafficabilityMatrix();
  double getTotalCost(base::Waypoint wInt);

  // -- node-level access (src/DyMu.hpp:500-518); std::nullopt = the reference's NULL --
  std::optional<globalNode> getGlobalNode(unsigned i, unsigned j);
  std::optional<globalNode> getNearestGlobalNode(base::Pose2D pos);
  std::optional<globalNode> getNearestGlobalNode(base::Waypoint wPos);
  std::optional<globalNode> globalGoal();  // the reference's public global_goal
  bool isSafeNode(unsigned i, unsigned j);         // :410-422 (border -> false)
  bool isFullyClosedNode(unsigned i, unsigned j);  // :424-436 (border -> false)
  void resetTotalCostMap();                        // :473-485: every node OPEN at +inf
  // the reference's global_narrowband (:445) as the last computeTotalCostMap left
  // it: snapshots of the band nodes in the reference's insertion order (rebuilt from
  // the values, csrc/pop_order.hpp); empty after computeEntireTotalCostMap
  std::vector<globalNode> globalNarrowband();
  // :548-567: the band node with the lowest total cost (first in insertion order
  // on ties), removed from the band list like the reference's erase; the map is
  // not changed.  std::nullopt on an empty band (the reference reads front()).
  std::optional<globalNode> minCostGlobalNode();
  // :487-498: the band holds only the goal (total cost 0)
  void resetGlobalNarrowBand();
  // :500-546: the reference update of node (i, j) from its nb4's current total costs
  // (a NULL neighbour: the other one alone; C from the node's cost, hazard and
  // trafficability); a lower value is taken, and a node whose total cost was +inf
  // joins the band (appended: insertion order, like the reference's vector) and the
  // propagated list.  Host arithmetic on the host copy of the map: for callers that
  // drive the propagation node by node; the solves run on the GPU.
  void propagateGlobalNode(unsigned i, unsigned j);
  void propagateGlobalNode(const globalNode& n);
  // the reference's public globalNode::state written by a caller (its FMM loop sets
  // CLOSED after each minCostGlobalNode); the next solve recomputes every state
  void setGlobalNodeState(unsigned i, unsigned j, node_state s);
  // global_propagated_nodes (:447): every node with a finite total cost in the
  // reference's insertion order, then those added by propagateGlobalNode.  (At 16384^2
  // after a full solve that is ~2.6e8 snapshots: globalPropagatedCount first.)
  std::vector<globalNode> globalPropagatedNodes();
  // the same list as grid indices (j * nx + i), without the snapshots
  std::vector<uint64_t> globalPropagatedIndices();
  uint64_t globalPropagatedCount();
  // every node's state (ny*nx, row-major: 1 CLOSED, 0 OPEN) as the last solve or the
  // caller's setGlobalNodeState left it (the reference's globalNode::state, in bulk)
  void copyNodeStates(uint8_t* out);
  // :731-784 / L:979-1023: the normalised descent direction at a node (the
  // reference's gradientNode(globalNode*) / gradientNode(localNode*))
  void gradientNode(unsigned i, unsigned j, double& dnx, double& dny) const;
  void gradientNode(const globalNode& n, double& dnx, double& dny) const;
  void gradientNode(const localNode& n, double& dnx, double& dny) const;

  // -- local layer (src/DyMu.hpp:539-591) --
  bool computeLocalPlanning(base::Waypoint wPos, base::samples::frame::Frame traversabilityMap,
                            double res, std::vector<base::Waypoint>& trajectory,
                            base::Time& localTime);
  int repairPath(base::Waypoint wInit, unsigned index);
  bool evaluatePath(unsigned starting_index);
  void expandRisk();
  // the set node, or std::nullopt (the reference's NULL; also after the
  // wall-clock limit, 5 s as in src/DyMu_LocalPathRepairing.cpp:685-696)
  std::optional<localNode> computeLocalPropagation(base::Waypoint wInit, base::Waypoint wOvertake);
  std::vector<base::Waypoint> getLocalPath(const localNode& lSetNode, base::Waypoint wInit,
                                           double tau);
  bool computeLocalWaypointGDM(base::Waypoint& wPos, double tau);
  std::optional<localNode> getLocalNode(base::Waypoint wPos);  // subdivides, like :177-189
  std::optional<localNode> getLocalNode(base::Pose2D pos);     // :160-173
  void subdivideGlobalNode(unsigned i, unsigned j);            // :150-156
  void createLocalMap(unsigned i, unsigned j);                 // :97-148 (as subdivide)
  // L:851-869: the step toward the nb4 sub-cell of lowest deviation
  base::Waypoint computeLocalWaypointDijkstra(const localNode& lNode);
  // the per-node steps of expandRisk / computeLocalPropagation (L:525-576, L:700-805):
  // maxRiskNode pops local_expandable_obstacles by the reference's rule (the front,
  // unless it is below 1 and a later entry is higher: then the first such), nullopt
  // when empty; propagateRisk / propagateLocalNode apply the risk / deviation update
  // to a sub-cell and queue it like the reference; minCostLocalNode pops the band
  // node of lowest deviation (SWEEPING, :752-775) or deviation + distance to
  // reachNode (CONSERVATIVE, :777-805), first strict minimum in insertion order
  // the reference's localNode::nb4List[d] (src/DyMu.hpp:52; d: 0 (i,j-1), 1 (i-1,j),
  // 2 (i+1,j), 3 (i,j+1)): nullopt where the reference holds NULL
  std::optional<localNode> localNeighbour(const localNode& n, int d);
  std::optional<localNode> maxRiskNode();
  // the reference's public localNode::state written by a caller (its loop closes each
  // popped node, L:654)
  void setLocalNodeState(const localNode& n, node_state s);
  void propagateRisk(const localNode& n);
  void propagateLocalNode(const localNode& n);
  std::optional<localNode> minCostLocalNode(double Tovertake, double minC);
  std::optional<localNode> minCostLocalNode(const localNode& reachNode);
  // the reference's public local lists (src/DyMu.hpp:448-454) as snapshots, in their
  // order: local_narrowband (insertion order), local_expandable_obstacles (queue
  // order), local_propagated_nodes (insertion order)
  std::vector<localNode> localNarrowband();
  std::vector<localNode> localExpandableObstacles();
  std::vector<localNode> localPropagatedNodes();
  // L:441-471 against current_path
  bool isBlockingObstacle(const localNode& obNode, unsigned& maxIndex, unsigned& minIndex);
  // the reference's local_agent (src/DyMu.hpp:460): the last local propagation's
  // start sub-cell, std::nullopt before one ran
  std::optional<localNode> localAgent();
  double getTotalCost(const localNode& lNode);                 // :473-491
  std::vector<std::vector<double>> getRiskMatrix(base::Waypoint rover_pos);
  std::vector<std::vector<double>> getDeviationMatrix(base::Waypoint rover_pos);
  int getReconnectingIndex();

  // -- extensions (not in the reference) --
  // computeLocalPropagation's wall-clock limit in seconds (the reference's fixed
  // 5.0, :685-696); <= 0 disables it
  void setLocalPropagationTimeout(double seconds) { local_timeout_s_ = seconds; }
  double localPropagationTimeout() const { return local_timeout_s_; }
  // Flat row-major views for FFI callers (ny*nx, index j*nx + i).  The total
  // cost lives on the device; this downloads whatever the host copy lacks.
  const double* totalCostData() const;
  // The whole total cost into out (ny*nx): raw (+inf unreachable) or as
  // getTotalCostMatrix (-1), row ranges on the host threads.
  void copyTotalCost(double* out, bool raw) const;
  unsigned sizeX() const { return nx_; }
  unsigned sizeY() const { return ny_; }
  bool hasGoal() const { return has_goal_; }
  unsigned goalI() const { return goal_i_; }
  unsigned goalJ() const { return goal_j_; }
  const dymu_stats& lastStats() const { return stats_; }
  // How the last computeTotalCostMap / computeEntireTotalCostMap ran: 0 cold
  // solve, 1 windowed re-propagation from the changed speed window, 2 map reused.
  int lastSolveKind() const { return incremental_; }
  // Local-layer feedback on the global layer (the writes of
  // src/DyMu_LocalPathRepairing.cpp:264-274 and :389-394), row-major ny*nx.
  // Only the rows that differ from the current values are re-packed and
  // uploaded before the next solve.
  bool setHazardDensity(const std::vector<double>& hd);
  bool setTrafficability(const std::vector<double>& tr);
  // Windowed forms: w x h values (row-major) for cells [i0, i0+w) x [j0, j0+h).
  bool setHazardDensityWindow(unsigned i0, unsigned j0, unsigned w, unsigned h,
                              const double* hd);
  bool setTrafficabilityWindow(unsigned i0, unsigned j0, unsigned w, unsigned h,
                               const double* tr);
  // Narrow-band cells left by the last computeTotalCostMap (0 after a full solve).
  uint64_t lastBandSize() const { return band_cells_.size(); }
  // How the last computeTotalCostMap resolved the reference's order at its exit
  // value: cells of exactly that value, how many of them the
  // reference had not closed yet, whether the exact host replay ran (degenerate
  // ties only), host time of the resolution and band replay.
  struct EarlyExitInfo {
    uint64_t tied = 0, open_at_limit = 0;
    int exact_replay = 0;         // 1: the exit was replayed exactly on the host
    double resolve_ms = 0.0;
    uint64_t replay_updates = 0;  // reference updates the band replay evaluated
    int band_exact = 1;           // every band value is the reference's (always, since round 6)
    // comparisons of engine values rounding could flip (near ties, pop_order.hpp's
    // TieGuard): any sends the exit to the exact host replay
    uint64_t near_ties = 0;
    unsigned replay_threads = 0;  // host threads of the band replay
  };
  const EarlyExitInfo& lastEarlyExitInfo() const { return early_info_; }
  // Engine options (device ordinal etc.); takes effect on the next solve.
  void setEngineOptions(const dymu_opts& o);
  // Install a total-cost map (ny*nx, +inf unreachable) as the state a
  // converged computeEntireTotalCostMap leaves: every finite node CLOSED (the
  // reference's public globalNode::total_cost / state writes).  The next
  // solve starts cold.  No solve runs here.
  bool loadTotalCostMap(const double* T);
  // local-layer inspection: how many global nodes are subdivided (mask: ny*nx
  // bytes, may be null), and one subdivided node's sub-cells (r*r each,
  // row-major) -- false if (i, j) has no local map
  uint64_t localMapMask(uint8_t* mask) const;
  bool localBlock(unsigned i, unsigned j, double* dev, double* tc, double* risk, uint8_t* state,
                  uint8_t* obst) const;
  unsigned resRatio() const { return res_ratio_; }

 private:
  uint64_t idx(unsigned i, unsigned j) const { return (uint64_t)j * nx_ + i; }
  // total cost of cell k: the device map, fetched into the host mirror in blocks
  // of kBlk x kBlk cells on first read
  double T(uint64_t k) const;
  void fetchAll() const;
  // body(r0, r1) over row chunks of the total cost, each once it is in the host
  // mirror (a stale mirror downloads chunk k+1 while body runs on chunk k)
  template <class Body>
  void streamTotalCost(Body&& body) const;
  // the reference's node state: CLOSED iff popped by its FMM (finite T not above
  // the last early-exit limit; every finite cell after a full solve)
  bool closedCell(uint64_t k) const;
  // node states written by a caller (setGlobalNodeState, resetTotalCostMap): empty =
  // derived from the last solve (closedCell's rule), else 1 = CLOSED per node
  std::vector<uint8_t> node_state_;
  void materializeStates();
  // nodes propagateGlobalNode made finite (global_propagated_nodes beyond the map's)
  std::vector<uint64_t> propagated_extra_;
  bool manual_list_ = false;  // after resetTotalCostMap: the list is propagated_extra_ alone
  // local per-node helpers (csrc/local_layer.cpp)
  void riskUpdate(uint64_t q);
  void deviationUpdate(uint64_t q);
  int64_t localId(const localNode& n) const;
  void markDirty(unsigned j0, unsigned j1);
  void ensureEngine();
  // pack F for the dirty rows, upload the rows whose speed changed; returns false
  // when nothing changed, else the bounding box of the changed cells
  bool syncSpeed(unsigned& i0, unsigned& i1, unsigned& j0, unsigned& j1);
  template <class ERows, class TRows>
  bool costMapFromRows(const ERows& elev_row, const TRows& terr_row);
  bool propagate(bool early, unsigned si, unsigned sj);
  // the band's tentative values at the moment `last` was popped; true when they are
  // not to be used: the reference's pop order was undetermined or near-tied (guard),
  // or the replay hit its work bound
  bool replayBand(uint64_t last, const std::vector<uint64_t>& band, std::vector<double>& out,
                  TieGuard& guard);
  // the reference's early exit replayed exactly on the host over the region box
  // (inclusive; empty: the whole grid) -- when the values cannot decide the exit
  bool exactEarlyExit(unsigned si, unsigned sj, const int64_t box[4]);
  // the reference FMM on the host (exact): until (si, sj) and its nb4 are CLOSED, or
  // the band empties for si < 0; over a box (inclusive, grown to the grid if short)
  struct HostFmm {
    int64_t bx[4], W = 0, PW = 0;
    std::vector<double> T;        // the box with a one-cell ring (+inf), row pitch PW
    std::vector<uint8_t> st;      // 1 CLOSED, 2 in the band (ring: 3 off the box, 4 off the grid)
    uint64_t at(int64_t i, int64_t j) const {  // grid cell (i, j) inside the box
      return (uint64_t)(j - bx[1] + 1) * (uint64_t)PW + (uint64_t)(i - bx[0] + 1);
    }
    std::vector<uint64_t> order;  // grid indices, in first-insertion order
    uint64_t band = 0;
  };
  HostFmm hostFmm(int64_t si, int64_t sj, const int64_t box[4]) const;
  // global_propagated_nodes' order after a GPU solve (reference insertion order)
  std::vector<uint64_t> insertionOrder();
  bool have_start_ = false;  // the last early exit's start and region (exact fallback)
  unsigned start_i_ = 0, start_j_ = 0;
  int64_t exit_box_[4] = {0, 0, -1, -1};
  double exit_r_const_ = 0.0;  // the constant-speed radius around the goal (TieGuard)
  // true once minCostGlobalNode checked the band's values for near ties (or the band
  // is exact / caller-built)
  bool band_values_checked_ = true;
  void settleBand();  // the check, and the exact replay on a near tie
  static constexpr uint64_t kReplayBudget = 1ull << 26;  // band-replay updates per exit
  static constexpr double kTieEps = 1e-12;        // near-tie bound (relative, TieGuard)
  static constexpr double kRegionMargin = 1e-9;   // the exit region: T <= t_closed (1 + this)
  // the host mirror's values for PopOrder
  struct MapT {
    const DyMuPathPlanner* p;
    double operator()(uint64_t k) const { return p->T(k); }
  };
  // band_cells_ into the reference's insertion order, if still in grid order
  void orderBand();
  bool safeNode(unsigned i, unsigned j) const;
  std::optional<globalNode> snapshot(uint64_t k);
  void nominalCost(unsigned i, unsigned j, int range, int num_locs, double cmax);
  // local layer internals (csrc/local_layer.cpp)
  int64_t nearestIndex(double x, double y) const;
  uint64_t localCell(uint64_t p, localNode* out) const;
  int64_t localAt(double x, double y);  // getLocalNode by sub-cell id, -1 = NULL
  double localTotalCost(uint64_t p) const;
  bool isBlockingObstacle(uint64_t p, unsigned& maxIndex, unsigned& minIndex,
                          const PathIndex* index = nullptr) const;
  int64_t localPropagation(base::Waypoint wInit, base::Waypoint wOvertake);
  std::vector<base::Waypoint> localPath(uint64_t set, base::Waypoint wInit);
  base::Waypoint dijkstraStep(uint64_t l) const;
  void windowMatrix(base::Waypoint rover_pos, bool deviation, std::vector<std::vector<double>>& m);

  static constexpr unsigned kBlk = 128;

  // parameters (src/DyMu.hpp:399-427)
  double risk_distance_, reconnect_distance_, risk_ratio_;
  repairingAproach repairing_approach_;
  unsigned nx_ = 0, ny_ = 0;
  double global_res_ = 1.0, local_res_ = 1.0;
  double local_timeout_s_ = 5.0;
  int64_t local_agent_ = -1;         // local_agent (sub-cell id), -1 = NULL
  unsigned res_ratio_ = 1;
  std::unique_ptr<LocalLayer> local_;
  std::vector<double> global_offset_{0.0, 0.0};
  std::vector<double> slope_range_;
  std::vector<std::string> locomotion_modes_;

  // SoA node fields (globalNode, src/DyMu.hpp:69-108)
  std::vector<double> elevation_, slope_, raw_cost_, cost_, hazard_, traff_;
  std::vector<uint32_t> terrain_;
  std::vector<uint8_t> is_obstacle_;
  std::vector<int32_t> loc_mode_;  // -1 = "DONT_CARE"

  bool has_goal_ = false;
  unsigned goal_i_ = 0, goal_j_ = 0;
  double goal_heading_ = 0.0;

  // engine and its device-resident map (pitch nx_)
  dymu_ctx* ctx_ = nullptr;
  dymu_opts opts_{-1, 0, 0, 0, 0, 0, 0, 0, 0};
  dymu_stats stats_{};
  double* dF_ = nullptr;
  double* dT_ = nullptr;
  uint64_t dcells_ = 0;
  // host mirror of dT_
  mutable std::vector<double> total_cost_;
  mutable std::vector<uint8_t> blk_ok_;  // read / written with atomic builtins (T())
  mutable uint64_t blk_missing_ = 0;
  mutable std::mutex fetch_mu_;          // T(): one block download at a time
  unsigned nbx_ = 0, nby_ = 0;
  void* registered_ = nullptr;  // total_cost_ buffer page-locked for DMA
  double closed_limit_ = 0.0;   // CLOSED iff finite T <= closed_limit_ ...
  // ... except these cells of exactly closed_limit_ (sorted): the reference's early
  // exit came before it popped them
  std::vector<uint64_t> open_at_limit_;
  std::vector<uint64_t> band_cells_;  // global_narrowband: grid indices
  bool band_unordered_ = false;       // band_cells_ in grid order until orderBand()
  EarlyExitInfo early_info_{};
  // F as uploaded to dF_ (host copy); node-field rows [dirty_j0_, dirty_j1_)
  // changed since it was packed
  std::vector<double> speed_;
  std::vector<double> row_;
  bool speed_valid_ = false;
  bool decrease_only_ = false;  // the last syncSpeed changed no speed upwards
  unsigned dirty_j0_ = 0, dirty_j1_ = 0;
  bool solved_ = false;  // dT_ holds the converged map of speed_ for the goal below
  unsigned solved_gi_ = 0, solved_gj_ = 0;
  int incremental_ = 0;  // last solve: 0 cold, 1 windowed re-propagation, 2 reused
};

}  // namespace PathPlanning_lib
