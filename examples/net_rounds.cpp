// net_rounds -- a multi-GPU network driven through the C ABI alone (gs_net_*,
// include/safe_gossip.h): what a host without Python --
// the reference's Rust crate over its FFI -- does to run node shards or rumor
// slices.  The reference harness's loop (src/gossiper.rs:173-259): inject
// every rumor at its origin, run rounds until no live push (`processed`,
// :209-212), report Statistics and the spread.
//
//   net_rounds --mode shards|slices [--transport rccl|local] [--world W]
//              [--rank g --id-file F] [--parts P] [--nodes n] [--rumors R]
//              [--seed S] [--epoch E] [--churn p] [--drop-push p]
//              [--drop-pull p] [--schedule 2P|SEQ] [--rounds K] [--device d]
//              [--dump FILE] [--time K]
//
// RCCL ranks (one process per GPU): rank 0 writes the RCCL id to --id-file,
// the others read it.  --dump writes, after every round, the round number,
// the network's any-live flag, every node's state codes (n*R u16,
// gs_dump_state's) and Statistics (n*5 u64) -- the whole network, from rank
// 0 -- so a checker can compare each round with another implementation.
// --time K: instead, after 3 unreported rounds, time K unreported rounds
// (nothing waits on the host between them) and print ms per round.
#include <safe_gossip.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static void die(const char *what, gs_status s) {
    std::fprintf(stderr, "net_rounds: %s: %s (status %d)\n", what, gs_status_string(s), (int)s);
    std::exit(1);
}

static uint32_t threshold(double p) {
    const double v = p * 4294967296.0 + 0.5;
    return v >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)v;
}

int main(int argc, char **argv) {
    std::string mode = "slices", transport = "rccl", id_file, dump, sched = "2P";
    uint32_t world = 1, rank = 0, parts = 4, n = 4096, R = 16, epoch = 0, rounds = 200, timed = 0;
    uint64_t seed = 0x5AFE6055ull;
    double churn = 0, dpush = 0, dpull = 0;
    int device = 0;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i], v = argv[i + 1];
        if (k == "--mode") mode = v;
        else if (k == "--transport") transport = v;
        else if (k == "--world") world = (uint32_t)std::stoul(v);
        else if (k == "--rank") rank = (uint32_t)std::stoul(v);
        else if (k == "--id-file") id_file = v;
        else if (k == "--parts") parts = (uint32_t)std::stoul(v);
        else if (k == "--nodes") n = (uint32_t)std::stoul(v);
        else if (k == "--rumors") R = (uint32_t)std::stoul(v);
        else if (k == "--seed") seed = std::stoull(v, nullptr, 0);
        else if (k == "--epoch") epoch = (uint32_t)std::stoul(v);
        else if (k == "--churn") churn = std::stod(v);
        else if (k == "--drop-push") dpush = std::stod(v);
        else if (k == "--drop-pull") dpull = std::stod(v);
        else if (k == "--schedule") sched = v;
        else if (k == "--rounds") rounds = (uint32_t)std::stoul(v);
        else if (k == "--device") device = std::stoi(v);
        else if (k == "--dump") dump = v;
        else if (k == "--time") timed = (uint32_t)std::stoul(v);
        else {
            std::fprintf(stderr, "net_rounds: unknown option %s\n", k.c_str());
            return 2;
        }
    }
    if (gs_abi_version() != GS_ABI_VERSION) {
        std::fprintf(stderr, "net_rounds: library ABI %u, header %u\n", gs_abi_version(), GS_ABI_VERSION);
        return 1;
    }
    gs_config cfg{};
    cfg.n_nodes = n;
    cfg.n_rumors = R;
    cfg.seed = seed;
    cfg.epoch = epoch;
    cfg.schedule = sched == "SEQ" ? GS_SCHED_SEQ : GS_SCHED_2P;
    cfg.device = device;
    cfg.churn = threshold(churn);
    cfg.drop_push = threshold(dpush);
    cfg.drop_pull = threshold(dpull);
    const gs_net_mode m = mode == "shards" ? GS_NET_SHARDS : GS_NET_SLICES;

    gs_net *net = nullptr;
    gs_status st;
    if (transport == "local") {
        st = gs_net_create_local(&cfg, m, world, parts, &net);
    } else {
        uint8_t id[GS_NET_ID_BYTES];
        if (rank == 0) {
            st = gs_net_unique_id(id);
            if (st != GS_OK) die("gs_net_unique_id", st);
            if (!id_file.empty()) {
                const std::string tmp = id_file + ".tmp";
                FILE *f = std::fopen(tmp.c_str(), "wb");
                if (!f || std::fwrite(id, 1, sizeof(id), f) != sizeof(id) || std::fclose(f) != 0) return 1;
                std::rename(tmp.c_str(), id_file.c_str());
            }
        } else {
            FILE *f = nullptr;
            for (int t = 0; t < 600 && !(f = std::fopen(id_file.c_str(), "rb")); ++t)
                std::this_thread::sleep_for(std::chrono::milliseconds(100));
            if (!f || std::fread(id, 1, sizeof(id), f) != sizeof(id)) return 1;
            std::fclose(f);
        }
        st = gs_net_create(&cfg, m, rank, world, parts, id, &net);
    }
    if (st != GS_OK) die("gs_net_create", st);

    for (uint32_t r = 0; r < R; ++r) {
        st = gs_net_send_new(net, gs_origin(seed, epoch, r, n), r);
        if (st != GS_OK) die("gs_net_send_new", st);
    }
    if (timed) {  // throughput: unreported rounds, one host wait at the end
        for (int w = 0; w < 3; ++w)
            if ((st = gs_net_next_round(net, nullptr)) != GS_OK) die("gs_net_next_round", st);
        if ((st = gs_net_sync(net)) != GS_OK) die("gs_net_sync", st);
        const auto a = std::chrono::steady_clock::now();
        for (uint32_t k = 0; k < timed; ++k)
            if ((st = gs_net_next_round(net, nullptr)) != GS_OK) die("gs_net_next_round", st);
        if ((st = gs_net_sync(net)) != GS_OK) die("gs_net_sync", st);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
        if (rank == 0)
            std::printf("{\"mode\": \"%s\", \"transport\": \"%s\", \"world\": %u, \"nodes\": %u, \"rumors\": %u, "
                        "\"parts\": %u, \"rounds\": %u, \"ms_per_round\": %.4f}\n",
                        mode.c_str(), transport.c_str(), world, n, R, parts, timed, ms / timed);
        gs_net_destroy(net);
        return 0;
    }
    FILE *df = nullptr;
    if (!dump.empty() && rank == 0 && !(df = std::fopen(dump.c_str(), "wb"))) return 1;
    std::vector<uint16_t> codes(dump.empty() ? 0 : (size_t)n * R);
    std::vector<uint64_t> stats(dump.empty() ? 0 : (size_t)n * 5);
    gs_round_report rep{};
    uint32_t full_round = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 0; k < rounds; ++k) {
        st = gs_net_next_round(net, &rep);
        if (st != GS_OK) die("gs_net_next_round", st);
        if (!dump.empty()) {
            if ((st = gs_net_dump_state(net, codes.data())) != GS_OK) die("gs_net_dump_state", st);
            if ((st = gs_net_statistics_all(net, stats.data())) != GS_OK) die("gs_net_statistics_all", st);
            if (df) {
                const uint32_t head[2] = {rep.round, rep.any_live};
                std::fwrite(head, sizeof(head), 1, df);
                std::fwrite(codes.data(), sizeof(uint16_t), codes.size(), df);
                std::fwrite(stats.data(), sizeof(uint64_t), stats.size(), df);
            }
        }
        if (!full_round) {
            uint64_t known = 0, complete = 0;
            if ((st = gs_net_known_counts(net, &known, &complete)) != GS_OK) die("gs_net_known_counts", st);
            if (complete == n) full_round = rep.round;
        }
        if (!rep.any_live) break;
    }
    if ((st = gs_net_sync(net)) != GS_OK) die("gs_net_sync", st);
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t known = 0, complete = 0;
    if ((st = gs_net_known_counts(net, &known, &complete)) != GS_OK) die("gs_net_known_counts", st);
    if (df) std::fclose(df);
    if (rank == 0)
        std::printf("{\"mode\": \"%s\", \"transport\": \"%s\", \"world\": %u, \"engines_here\": %u, \"rounds\": %u, "
                    "\"round_full\": %u, \"known\": %llu, \"complete\": %llu, \"seconds\": %.3f}\n",
                    mode.c_str(), transport.c_str(), world, gs_net_local_engines(net), rep.round, full_round,
                    (unsigned long long)known, (unsigned long long)complete, secs);
    gs_net_destroy(net);
    return 0;
}
