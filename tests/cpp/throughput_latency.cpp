// Restatement of the reference's throughput/latency experiment driver
// (experiments/src/throughput-latency.cpp:3-194) written against the
// reference API only: it includes <wharfmh.h> and uses config::, types::,
// dygrl::WharfMH, utility::generate_batch_of_edges, read_unweighted_graph,
// pbbs:: and the config.h update timers exactly as a reference driver does.
// Built with -I include/compat (include/compat/wharfmh.h), so the only
// difference from building it against the reference is the include path.
// tests/test_cpp_dropin.py compiles it on the CPU and runs it on the GPU.
#include <wharfmh.h>

static void set_model(const string& model, double p, double q)
{
    if (model == "deepwalk") {
        config::random_walk_model = types::RandomWalkModelType::DEEPWALK;
        std::cout << "Walking model: DEEPWALK" << std::endl;
    } else if (model == "node2vec") {
        config::random_walk_model = types::RandomWalkModelType::NODE2VEC;
        config::paramP = p;
        config::paramQ = q;
        std::cout << "Walking model: NODE2VEC | Params (p,q) = (" << config::paramP << "," << config::paramQ << ")"
                  << std::endl;
    } else {
        std::cerr << "Unrecognized walking model! Abort" << std::endl;
        std::exit(1);
    }
}

static void set_init(const string& init)
{
    if (init == "burnin") config::sampler_init_strategy = types::SamplerInitStartegy::BURNIN;
    else if (init == "weight") config::sampler_init_strategy = types::SamplerInitStartegy::WEIGHT;
    else if (init == "random") config::sampler_init_strategy = types::SamplerInitStartegy::RANDOM;
    else {
        std::cerr << "Unrecognized sampler init strategy" << std::endl;
        std::exit(1);
    }
    std::cout << "Sampler strategy: " << init << std::endl;
}

static void print_latencies(const char* what, const pbbs::sequence<double>& lat)
{
    std::cout << "Average walk " << what << " latency = { ";
    for (size_t t = 0; t < lat.size(); t++) std::cout << lat[t] << " ";
    std::cout << "}" << std::endl;
}

void throughput(commandLine& P)
{
    const string fname = string(P.getOptionValue("-f", default_file_name));
    const bool mmap = P.getOption("-m");
    const bool is_symmetric = P.getOption("-s");
    const size_t wpv = P.getOptionLongValue("-w", config::walks_per_vertex);
    const size_t len = P.getOptionLongValue("-l", config::walk_length);
    const string model = string(P.getOptionValue("-model", "deepwalk"));
    const double paramP = P.getOptionDoubleValue("-paramP", config::paramP);
    const double paramQ = P.getOptionDoubleValue("-paramQ", config::paramQ);
    const string init = string(P.getOptionValue("-init", "weight"));
    const size_t n_trials = P.getOptionLongValue("-trials", 3);
    const string det = string(P.getOptionValue("-det", "true"));
    const size_t max_batch = P.getOptionLongValue("-maxbatch", 500);

    config::walks_per_vertex = wpv;
    config::walk_length = len;
    std::cout << "Walks per vertex: " << (int)config::walks_per_vertex << std::endl;
    std::cout << "Walk length: " << (int)config::walk_length << std::endl;
    set_model(model, paramP, paramQ);
    set_init(init);
    config::deterministic_mode = det == "true";
    cout << "determinism=" << config::deterministic_mode << endl;

    size_t n, m;
    uintE* offsets;
    uintV* edges;
    std::tie(n, m, offsets, edges) = read_unweighted_graph(fname.c_str(), is_symmetric, mmap);

    dygrl::WharfMH WharfMH = dygrl::WharfMH(n, m, offsets, edges);   // takes over (frees) the arrays
    WharfMH.generate_initial_random_walks();

    auto batch_sizes = pbbs::sequence<size_t>();
    for (size_t b = 5; b <= max_batch; b *= 10) batch_sizes.push_back(b);

    for (size_t i = 0; i < batch_sizes.size(); i++) {
        timer insert_timer("InsertTimer", false);
        timer delete_timer("DeleteTimer", false);
        graph_update_time_on_insert.reset();
        walk_update_time_on_insert.reset();
        graph_update_time_on_delete.reset();
        walk_update_time_on_delete.reset();

        std::cout << std::endl << "Batch size = " << 2 * batch_sizes[i] << " | ";
        double prev_insert = 0, prev_delete = 0;
        auto latency_insert = pbbs::sequence<double>(n_trials);
        auto latency_delete = pbbs::sequence<double>(n_trials);
        auto latency = pbbs::sequence<double>(n_trials);
        double affected_insert = 0, affected_delete = 0;

        for (size_t trial = 0; trial < n_trials; trial++) {
            const size_t graph_size_pow2 = 1 << (pbbs::log2_up(n) - 1);
            auto batch = utility::generate_batch_of_edges(batch_sizes[i], n, false, false);
            std::cout << batch.second << " ";

            insert_timer.start();
            auto x = WharfMH.insert_edges_batch(batch.second, batch.first, false, true, graph_size_pow2);
            insert_timer.stop();
            affected_insert += x.size();
            const double ins = walk_update_time_on_insert.get_total() - prev_insert;
            prev_insert = ins;
            latency_insert[trial] = ins / std::max<size_t>(x.size(), 1);

            delete_timer.start();
            auto y = WharfMH.delete_edges_batch(batch.second, batch.first, false, true, graph_size_pow2);
            delete_timer.stop();
            affected_delete += y.size();
            const double del = walk_update_time_on_delete.get_total() - prev_delete;
            prev_delete = del;
            latency_delete[trial] = del / std::max<size_t>(y.size(), 1);
            latency[trial] = (ins + del) / std::max<size_t>(x.size() + y.size(), 1);

            pbbs::free_array(batch.first);
        }
        std::cout << std::endl;
        std::cout << "Average insert time = " << insert_timer.get_total() / n_trials << std::endl;
        std::cout << "Average graph update insert time = " << graph_update_time_on_insert.get_total() / n_trials
                  << std::endl;
        std::cout << "Average walk update insert time = " << walk_update_time_on_insert.get_total() / n_trials
                  << " | Average number of walks affected = " << affected_insert / n_trials << std::endl;
        std::cout << "Average delete time = " << delete_timer.get_total() / n_trials << std::endl;
        std::cout << "Average graph update delete time = " << graph_update_time_on_delete.get_total() / n_trials
                  << std::endl;
        std::cout << "Average walk update delete time = " << walk_update_time_on_delete.get_total() / n_trials
                  << " | Average number of walks affected = " << affected_delete / n_trials << std::endl;
        print_latencies("insert", latency_insert);
        print_latencies("delete", latency_delete);
        print_latencies("update", latency);
    }

    // deferred walk update: apply_walk_updates = false returns rewalk_points.size()
    // unfilled entries (wharfmh.h:547-548); batch_walk_update applies them later
    {
        auto batch = utility::generate_batch_of_edges(50, n, 7, false, false);
        auto z = WharfMH.insert_edges_batch(batch.second, batch.first, false, true,
                                            std::numeric_limits<size_t>::max(), false);
        std::vector<types::Vertex> sources;
        for (size_t e = 0; e < batch.second; e++) sources.push_back(std::get<0>(batch.first[e]));
        auto applied = WharfMH.batch_walk_update(sources);
        std::cout << "Deferred walk update: " << z.size() << " rewalk points, " << applied.size()
                  << " walks updated" << (z.size() == applied.size() ? " (match)" : " (MISMATCH)") << std::endl;
        pbbs::free_array(batch.first);
    }

    WharfMH.destroy_index();
    timer generate_timer("Generate Initial Random Walks", false);
    for (size_t i = 0; i < n_trials; i++) {
        generate_timer.start();
        WharfMH.generate_initial_random_walks();
        generate_timer.stop();
        WharfMH.destroy_index();
    }
    std::cout << std::endl
              << "Average time to generate random walks from scratch = " << generate_timer.get_total() / n_trials
              << std::endl
              << std::endl;
}

int main(int argc, char** argv)
{
    std::cout << " - running throughput-latency experiment with " << num_workers() << " threads" << std::endl;
    commandLine P(argc, argv, "");
    throughput(P);
}
